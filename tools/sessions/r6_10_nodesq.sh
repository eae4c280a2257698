#!/bin/bash
# round 6, session 10: SQ counters (serial schedule, fused node layer = k_node_ws) and FETCH/WRITE
# passes for the node kernels' HBM bytes
set -e
TAG=_r6ws BENCH_EXTRA="--node-kernel fused" bash tools/counters.sh
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
B="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu --no-prologue --no-sub --complexes 32 --overlap 0 --node-kernel fused"
timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/r6_10_fetch -o run -- $B > /dev/null 2>&1
timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/r6_10_write -o run -- $B > /dev/null 2>&1
python3 $R/tools/sq_summary.py r6_10_traffic r6_10_fetch r6_10_write
