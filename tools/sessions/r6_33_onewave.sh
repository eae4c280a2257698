#!/bin/bash
# round 6, session 33: one store wave per CU (256 x 1) with a deeper store window (diag inflight6 /
# inflight4: the same stores in flight as 512 waves x 3) vs the product (256 x 2, window 3);
# interleaved, 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
L=deepinteract_amd/lib/variants
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_33_prod_$r.json
  timeout -k 10 240 python bench.py $B --pair-blocks 256 --pair-waves 1 --lib $L/diag_inflight6/libdeepinteract_amd.so > $O/r6_33_1w6_$r.json
  timeout -k 10 240 python bench.py $B --pair-blocks 256 --pair-waves 1 --lib $L/diag_inflight4/libdeepinteract_amd.so > $O/r6_33_1w4_$r.json
  timeout -k 10 240 python bench.py $B --pair-blocks 384 --pair-waves 1 --lib $L/diag_inflight4/libdeepinteract_amd.so > $O/r6_33_384w4_$r.json
  python tools/show_bench.py $O/r6_33_*_$r.json
done
