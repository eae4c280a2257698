#!/bin/bash
# round 4 v13: with the pair stream now the longer one (v12), a larger pair grid / deeper store bound
# beside GeoT (2 rounds)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=deepinteract_amd/lib/variants
L() { echo "--lib $V/$1/libdeepinteract_amd.so"; }
tools/ab.sh 2 "d|" "b144|--pair-blocks 144" "b160|--pair-blocks 160" "i4|$(L infl4)" "i5|$(L infl5)"
