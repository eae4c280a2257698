#!/bin/bash
# round 4 v8: chain-1 pair planes as contiguous whole-line runs (c1run: nt, c1run16: sc1) -- the pair
# parity tests against that build first, then the A/B vs the default (2 rounds)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=deepinteract_amd/lib/variants
L() { echo "--lib $V/$1/libdeepinteract_amd.so"; }
tools/gpu_run.sh "par_c1run:300:DI_TEST_VARIANT=$R/$V/c1run/libdeepinteract_amd.so python -u -m pytest tests/test_gpu_parity.py -k pair -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "par_c1run16:300:DI_TEST_VARIANT=$R/$V/c1run16/libdeepinteract_amd.so python -u -m pytest tests/test_gpu_parity.py -k pair -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" &&
tools/ab.sh 2 "x32|" "c1|$(L c1run)" "c116|$(L c1run16)"
