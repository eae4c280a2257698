# round 5: edge ring with dynamic tile tickets vs static tiles (variant statictiles)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
V=deepinteract_amd/lib/variants
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
timeout -k 10 400 python -u -m pytest -q -s --timeout 240 --timeout-method thread tests/test_gpu_edge_x32.py tests/test_gpu_c3.py tests/test_gpu_parity.py tests/test_gpu_fold.py > $O/g24_pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 150 python bench.py $B > $O/g24_dyn_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --lib $V/statictiles/libdeepinteract_amd.so > $O/g24_static_$r.json 2>/dev/null || exit 1
done
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 > $O/g24_ser_dyn.json 2>/dev/null || exit 1
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 --lib $V/statictiles/libdeepinteract_amd.so > $O/g24_ser_static.json 2>/dev/null
