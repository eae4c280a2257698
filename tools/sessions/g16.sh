# round 5: k_node_fast v2 (Q/K/V prefetch, <= 120 VGPRs) vs v1 (variant nf1); resident InitEdge + embed launch in the overlapped schedule
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
V=deepinteract_amd/lib/variants
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
timeout -k 10 300 python -u -m pytest -q -s --timeout 240 --timeout-method thread tests/test_gpu_node_aggr.py > $O/g16_pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 150 python bench.py $B > $O/g16_v2_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --lib $V/nf1/libdeepinteract_amd.so > $O/g16_v1_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --init-kernel split > $O/g16_v2split_$r.json 2>/dev/null || exit 1
done
timeout -k 10 300 python tools/diag/interference.py --only init,init_res,node0,node1 > $O/g16_interf.jsonl 2> $O/g16_interf.err
