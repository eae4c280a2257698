# round 5: InitEdge + embedding on the 8-wave ring (k_init_x32_ring) vs the staged k_init_x32 (variant initold)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
V=deepinteract_amd/lib/variants
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
timeout -k 10 400 python -u -m pytest -q -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_node_aggr.py tests/test_gpu_fold.py > $O/g21_pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 150 python bench.py $B > $O/g21_ring_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --lib $V/initold/libdeepinteract_amd.so > $O/g21_old_$r.json 2>/dev/null || exit 1
done
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 > $O/g21_ser_ring.json 2>/dev/null || exit 1
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 --lib $V/initold/libdeepinteract_amd.so > $O/g21_ser_old.json 2>/dev/null || exit 1
timeout -k 10 200 python tools/diag/interference.py --only init > $O/g21_interf.jsonl 2>/dev/null
