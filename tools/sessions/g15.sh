# round 5: k_node_fast (bf16 di_node_layer at full occupancy): parity, then A/B vs the previous tree (variant nodeold)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
V=deepinteract_amd/lib/variants
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
timeout -k 10 400 python -u -m pytest -q -s --timeout 240 --timeout-method thread tests/test_gpu_node_aggr.py tests/test_gpu_c3.py tests/test_gpu_parity.py tests/test_gpu_variants.py > $O/g15_pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 150 python bench.py $B > $O/g15_fast_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --lib $V/nodeold/libdeepinteract_amd.so > $O/g15_old_$r.json 2>/dev/null || exit 1
done
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 --node-kernel fused > $O/g15_ser_fast.json 2>/dev/null || exit 1
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 --node-kernel fused --lib $V/nodeold/libdeepinteract_amd.so > $O/g15_ser_old.json 2>/dev/null || exit 1
timeout -k 10 300 python tools/diag/interference.py > $O/g15_interf.jsonl 2> $O/g15_interf.err
