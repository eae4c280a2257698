#!/bin/bash
# round 6, session 39: the edge ring's blocks of one XCD kept within a tile of each other by a per-XCD
# tile barrier (diag xcdbar: fewer weight stages live in the XCD's L2 at once) vs the product;
# interleaved, 3 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_xcdbar/libdeepinteract_amd.so
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2 3; do
  timeout -k 10 240 python bench.py $B > $O/r6_39_prod_$r.json
  timeout -k 10 240 python bench.py $B --lib $V > $O/r6_39_xcdbar_$r.json
  python tools/show_bench.py $O/r6_39_*_$r.json
done
