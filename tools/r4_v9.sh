#!/bin/bash
# round 4 v9: chain-1 contiguous runs with the store bound every 2nd / 3rd store (parity first)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=deepinteract_amd/lib/variants
L() { echo "--lib $V/$1/libdeepinteract_amd.so"; }
tools/gpu_run.sh "par_b2:300:DI_TEST_VARIANT=$R/$V/c1runb2/libdeepinteract_amd.so python -u -m pytest tests/test_gpu_parity.py -k pair -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" &&
tools/ab.sh 2 "x32|" "b1|$(L c1run)" "b2|$(L c1runb2)" "b3|$(L c1runb3)"
