# round 5: timing diagnostics (tools/diag/patch_build.py) beside the pair stream and alone
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
V=deepinteract_amd/lib/variants
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
for r in 1 2; do
  for d in base diag_nosilu diag_nosync diag_w0; do
    L=""; [ $d != base ] && L="--lib $V/$d/libdeepinteract_amd.so"
    timeout -k 10 150 python bench.py $B $L > $O/g7_${d}_$r.json 2>/dev/null || exit 1
  done
done
for d in base diag_w0 diag_nosync; do
  L=""; [ $d != base ] && L="--lib $V/$d/libdeepinteract_amd.so"
  timeout -k 10 150 python bench.py $B --overlap 0 --complexes 256 $L > $O/g7_ser_${d}.json 2>/dev/null || exit 1
done
