# round 5: fold with its loads in flight beside K / Q: tests, A/B fused vs fold (overlapped, serial)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
timeout -k 10 300 python -u -m pytest -q -s --timeout 240 --timeout-method thread tests/test_gpu_fold.py > $O/g11_pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 150 python bench.py $B > $O/g11_fused_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --node-kernel fold > $O/g11_fold_$r.json 2>/dev/null || exit 1
done
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 > $O/g11_ser_split.json 2>/dev/null || exit 1
timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 --node-kernel fold > $O/g11_ser_fold.json 2>/dev/null
