#!/bin/bash
# round 4 v5 A/B: pair-store priority, lin32_pipe MFMA lead, edge-block priority, row loads after the
# stage barrier (2 rounds); timing diagnostics (no SiLU / no stage waits) and disjoint CU sets (1 round)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=deepinteract_amd/lib/variants
L() { echo "--lib $V/$1/libdeepinteract_amd.so"; }
tools/ab.sh 2 "x32|" "pp1|$(L pprio1)" "pp3|$(L pprio3)" "ld2|$(L lead2)" "ep|$(L eprio)" "rl|$(L rowld)" "df|$(L defer)" &&
tools/ab.sh 1 "ns|$(L nosilu)" "ny|$(L nosync)" "r0|$(L reread0)" "pc64|--pair-cus 64 --pair-blocks 64 --pair-waves 8"
