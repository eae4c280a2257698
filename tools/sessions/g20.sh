# round 5: k_node_fast with 2 node groups per block (product) vs 1 (ng1); edge ring 3 stages ahead (ahead3)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
V=deepinteract_amd/lib/variants
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
timeout -k 10 300 python -u -m pytest -q -s --timeout 240 --timeout-method thread tests/test_gpu_node_aggr.py tests/test_gpu_c3.py > $O/g20_pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 150 python bench.py $B > $O/g20_ng2_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --lib $V/diag_ng1/libdeepinteract_amd.so > $O/g20_ng1_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --lib $V/diag_ahead3/libdeepinteract_amd.so > $O/g20_ahead3_$r.json 2>/dev/null || exit 1
done
