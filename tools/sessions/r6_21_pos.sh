#!/bin/bash
# round 6, session 21: InitEdge's positional-row gathers at half their bytes (diag posh: what a bf16
# copy of the fp32 tables would gather) vs product vs none (initnopos): pair rate beside InitEdge
# (tools/diag/interference.py) and the step (2 interleaved rounds, C3 512 complexes)
set -e
O=gpurun_out; mkdir -p $O
L=deepinteract_amd/lib/variants
for v in product posh initnopos; do
  lib=""; [ $v != product ] && lib="--lib $L/diag_$v/libdeepinteract_amd.so"
  timeout -k 10 200 python tools/diag/interference.py --only init $lib > $O/r6_21_interf_$v.jsonl
  cat $O/r6_21_interf_$v.jsonl
done
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_21_prod_$r.json
  timeout -k 10 240 python bench.py $B --lib $L/diag_posh/libdeepinteract_amd.so > $O/r6_21_posh_$r.json
  python tools/show_bench.py $O/r6_21_*_$r.json
done
