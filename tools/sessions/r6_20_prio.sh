#!/bin/bash
# round 6, session 20: static issue priority / stagger A/B (tools/diag/patch_build.py prio47 prio03
# stag nodeprio pairprio prio47node) vs the product, interleaved, 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
L=deepinteract_amd/lib/variants
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_20_prod_$r.json
  for v in prio47 prio03 stag nodeprio pairprio prio47node; do
    timeout -k 10 240 python bench.py $B --lib $L/diag_$v/libdeepinteract_amd.so > $O/r6_20_${v}_$r.json
  done
  python tools/show_bench.py $O/r6_20_*_$r.json
done
