#!/bin/bash
# Pair-kernel variants: parity tests on the default build, then serial and overlapped timing per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_run.sh "pair_tests:300:python -u -m pytest tests/test_gpu_parity.py -k pair -x -q --timeout 120 --timeout-method thread" || exit 1
TAG=s tools/variants.sh "$@" && TAG=o BENCH_ARGS="--no-cpu --complexes 256 --steps 2 --warmup 1" tools/variants.sh "$@"
