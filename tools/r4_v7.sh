#!/bin/bash
# round 4 v7 A/B: whole-line pair stores (k_pair_lines, no partial lines) with nt vs sc1 / sc1 nt
# (write-through, dropped from L2) beside GeoT, vs the default row streaming (2 rounds)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=deepinteract_amd/lib/variants
L() { echo "--lib $V/$1/libdeepinteract_amd.so"; }
tools/ab.sh 2 "x32|" "ln|--pair-kernel lines" "ln16|--pair-kernel lines $(L cpol16)" "ln18|--pair-kernel lines $(L cpol18)"
