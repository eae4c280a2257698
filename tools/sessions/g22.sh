# round 5: pair-stream grid re-balanced against the faster GeoT (k_node_fast)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
for r in 1 2; do
  for pb in 128 112 144 160; do
    timeout -k 10 150 python bench.py $B --pair-blocks $pb > $O/g22_b${pb}_$r.json 2>/dev/null || exit 1
  done
done
