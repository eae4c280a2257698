# round 5: kernel trace of the pair-queue schedule + launch-shape variants (512 complexes, 3 steps)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/g2_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-sub --no-prologue --complexes 256 --steps 2 --warmup 1 > $O/g2_trace_bench.json 2> $O/g2_trace.err) && \
timeout -k 10 150 python bench.py $B > $O/g2_a.json 2>/dev/null && \
timeout -k 10 150 python bench.py $B --pair-blocks 256 --pair-waves 2 > $O/g2_b.json 2>/dev/null && \
timeout -k 10 150 python bench.py $B --ring 32 --help-every 8 > $O/g2_c.json 2>/dev/null && \
timeout -k 10 150 python bench.py $B > $O/g2_a2.json 2>/dev/null
