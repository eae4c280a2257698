#!/bin/bash
# round 6, session 38: the edge ring's weight stream at full bytes but an always-L2-hot footprint
# (diag ringw0) vs half the bytes (diag whalf) vs the product: is it the stream's L2 misses or its
# bytes that cost the pair stream? Interleaved, 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
L=deepinteract_amd/lib/variants
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_38_prod_$r.json
  timeout -k 10 240 python bench.py $B --lib $L/diag_ringw0/libdeepinteract_amd.so > $O/r6_38_ringw0_$r.json
  timeout -k 10 240 python bench.py $B --lib $L/diag_whalf/libdeepinteract_amd.so > $O/r6_38_whalf_$r.json
  python tools/show_bench.py $O/r6_38_*_$r.json
done
