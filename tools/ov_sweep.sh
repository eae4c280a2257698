#!/bin/bash
# Pair parity tests, then the overlap schedules x pair-kernel variants (tools/build_variants.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V="${*:-base}"
tools/gpu_run.sh "pair_tests:300:python -u -m pytest tests/test_gpu_parity.py -k pair -x -q --timeout 120 --timeout-method thread" || exit 1
for o in ${OVS:-1 2}; do
  TAG=o$o BENCH_ARGS="--no-cpu --complexes 256 --steps 2 --warmup 1 --overlap $o" tools/variants.sh $V || exit 1
done
