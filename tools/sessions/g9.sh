# round 5: rotating-issuer weight ring vs k_edge_x32 (variant ring0); parity incl. elementwise logits, C4
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
V=deepinteract_amd/lib/variants
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_edge_x32.py tests/test_gpu_c3.py tests/test_gpu_parity.py tests/test_gpu_modules.py tests/test_gpu_api.py tests/test_gpu_c4.py > $O/g9_pytest.log 2>&1
for r in 1 2; do
  timeout -k 10 150 python bench.py $B > $O/g9_ring_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --lib $V/ring0/libdeepinteract_amd.so > $O/g9_x32_$r.json 2>/dev/null || exit 1
done
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 > $O/g9_ser_ring.json 2>/dev/null || exit 1
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 --lib $V/ring0/libdeepinteract_amd.so > $O/g9_ser_x32.json 2>/dev/null
