# round 5: pair store window 4 (inflight4), help cadence 2 / 8, hT ring 32
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
V=deepinteract_amd/lib/variants
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
for r in 1 2; do
  timeout -k 10 150 python bench.py $B > $O/g23_base_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --lib $V/diag_inflight4/libdeepinteract_amd.so > $O/g23_inf4_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --help-every 2 > $O/g23_he2_$r.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py $B --help-every 8 --ring 32 > $O/g23_he8r32_$r.json 2>/dev/null || exit 1
done
