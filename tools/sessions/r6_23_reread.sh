#!/bin/bash
# round 6, session 23: the edge ring's F-row re-reads always L2-hot (diag reread0) vs the product,
# interleaved, 3 rounds, C3 512 complexes: the upper bound of keeping F rows on chip
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_reread0/libdeepinteract_amd.so
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2 3; do
  timeout -k 10 240 python bench.py $B > $O/r6_23_prod_$r.json
  timeout -k 10 240 python bench.py $B --lib $V > $O/r6_23_reread0_$r.json
  python tools/show_bench.py $O/r6_23_*_$r.json
done
