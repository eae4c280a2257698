#!/bin/bash
# round 4 v14: with the pair stream the longer one, plain (cpol 0) / sc0 (cpol 1) pair stores beside
# GeoT vs nt (2 rounds)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=deepinteract_amd/lib/variants
L() { echo "--lib $V/$1/libdeepinteract_amd.so"; }
tools/ab.sh 2 "nt|" "c0|$(L cpol0)" "c1|$(L cpol1)"
