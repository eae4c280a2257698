#!/bin/bash
# round 4 v10: contiguous chain-1 runs with the pair waves at s_setprio 3 (issue priority over the
# VALU-dense GeoT waves) vs the runs alone vs the default (2 rounds)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=deepinteract_amd/lib/variants
L() { echo "--lib $V/$1/libdeepinteract_amd.so"; }
tools/ab.sh 2 "x32|" "c1|$(L c1run)" "c1p3|$(L c1runp3)"
