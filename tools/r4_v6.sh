#!/bin/bash
# round 4 v6 A/B: pair stores beside GeoT as sc1 / sc0 sc1 / sc1 nt (dropped from L2) vs nt;
# deferred block-3 epilogues; the row re-read diagnostic (2 rounds)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=deepinteract_amd/lib/variants
L() { echo "--lib $V/$1/libdeepinteract_amd.so"; }
tools/ab.sh 2 "x32|" "c16|$(L cpol16)" "c17|$(L cpol17)" "c18|$(L cpol18)" "df|$(L defer)" "r0|$(L reread0)"
