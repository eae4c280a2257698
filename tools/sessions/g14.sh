# round 5: per-kernel interference with the pair stream; the --dist gather record
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python tools/diag/interference.py > $O/g14_interf.jsonl 2> $O/g14_interf.err || exit 1
timeout -k 10 400 python bench.py --dist --no-cpu --no-sub --no-prologue --complexes 256 --steps 2 --warmup 1 > $O/g14_dist.json 2> $O/g14_dist.err
