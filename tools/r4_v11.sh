#!/bin/bash
# round 4 v11: the edge row's lines touched one stage ahead of each re-read (pfetch) vs default (3 rounds)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=deepinteract_amd/lib/variants
L() { echo "--lib $V/$1/libdeepinteract_amd.so"; }
tools/ab.sh 3 "x32|" "pf|$(L pfetch)"
