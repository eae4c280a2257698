#!/bin/bash
# round 6, session 28: schedule parameters tuned in rounds 3-5 re-checked at the new pair-stream
# shape (one 2-wave block per CU): store window 2 / 4 (diag inflight2 / inflight4; product 3), help
# cadence 2 / 8 (product 4), micro-batch 16 (product 8), node layer folded into the edge layer;
# interleaved, 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
L=deepinteract_amd/lib/variants
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_28_prod_$r.json
  timeout -k 10 240 python bench.py $B --lib $L/diag_inflight2/libdeepinteract_amd.so > $O/r6_28_inflight2_$r.json
  timeout -k 10 240 python bench.py $B --lib $L/diag_inflight4/libdeepinteract_amd.so > $O/r6_28_inflight4_$r.json
  timeout -k 10 240 python bench.py $B --help-every 2 > $O/r6_28_help2_$r.json
  timeout -k 10 240 python bench.py $B --help-every 8 > $O/r6_28_help8_$r.json
  timeout -k 10 240 python bench.py $B --micro-batch 16 > $O/r6_28_mb16_$r.json
  timeout -k 10 240 python bench.py $B --node-kernel fold > $O/r6_28_fold_$r.json
  python tools/show_bench.py $O/r6_28_*_$r.json
done
