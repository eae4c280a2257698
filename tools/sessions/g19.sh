# round 5: what in InitEdge costs the pair stream its rate (diagnostic builds: wrong results, timing only)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
V=deepinteract_amd/lib/variants
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
timeout -k 10 200 python tools/diag/interference.py --only init > $O/g19_interf_base.jsonl 2>/dev/null || exit 1
for d in initnopos initnostore initw0; do
  timeout -k 10 200 python tools/diag/interference.py --only init --lib $V/diag_$d/libdeepinteract_amd.so > $O/g19_interf_$d.jsonl 2>/dev/null || exit 1
done
timeout -k 10 150 python bench.py $B > $O/g19_base.json 2>/dev/null || exit 1
for d in initnopos initnostore initw0; do
  timeout -k 10 150 python bench.py $B --lib $V/diag_$d/libdeepinteract_amd.so > $O/g19_$d.json 2>/dev/null || exit 1
done
