#!/bin/bash
# Sample the GPU's reported clocks / power while a bench runs (is the overlapped schedule
# power- or clock-limited?). usage: tools/clock_probe.sh <tag> <bench args...>
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
tag=$1; shift
out=gpurun_out/clk_${tag}.txt
: > $out
( for i in $(seq 1 200); do echo "t=$i" >> $out; timeout 5 rocm-smi --showclocks --showpower >> $out 2>&1; sleep 0.05; done ) &
sp=$!
timeout -k 10 200 python bench.py "$@" > gpurun_out/clk_${tag}.json
rc=$?
kill $sp 2>/dev/null; wait $sp 2>/dev/null
exit $rc
