# round 5: pair-stream launch granularity (jobs per launch) and grid, 512 complexes, 3 steps, 2 rounds
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
for r in 1 2; do
timeout -k 10 150 python bench.py $B > $O/g3_all$r.json 2>/dev/null && \
timeout -k 10 150 python bench.py $B --jobs-per-launch 1 > $O/g3_j1$r.json 2>/dev/null && \
timeout -k 10 150 python bench.py $B --jobs-per-launch 8 > $O/g3_j8$r.json 2>/dev/null && \
timeout -k 10 150 python bench.py $B --pair-blocks 160 > $O/g3_b160$r.json 2>/dev/null && \
timeout -k 10 150 python bench.py $B --pair-blocks 96 > $O/g3_b96$r.json 2>/dev/null || exit 1
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/g3_trace_j1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-sub --no-prologue --complexes 256 --steps 2 --warmup 1 --jobs-per-launch 1 > $O/g3_trace_j1.json 2>/dev/null
