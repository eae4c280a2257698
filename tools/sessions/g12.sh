# round 5: pair stream alone at the beside shapes; kernel trace of the default overlapped schedule; SQ passes (ring edge kernel)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python tools/diag/pair_alone.py > $O/g12_pair_alone.jsonl 2> $O/g12_pair_alone.err || exit 1
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/g12_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu --no-sub --no-prologue --complexes 256 > $O/g12_trace.json 2>/dev/null || exit 1
cd $GRAFT_REPO_ROOT && python tools/timeline.py $O/g12_trace/run_kernel_trace.csv --save $O/g12_timeline.csv > $O/g12_timeline.txt 2>&1
rm -f $O/g12_trace/run_kernel_trace.csv
TAG=_g12 bash tools/counters.sh
cd $GRAFT_REPO_ROOT && timeout -k 10 400 python bench.py --dist --no-cpu --no-sub --no-prologue --complexes 64 --steps 2 --warmup 1 > $O/g12_dist.json 2> $O/g12_dist.err
