#!/bin/bash
# round 6, session 29: A/B variants measured before the pair-stream shape change, re-run at the new
# shape (one 2-wave block per CU): edge ring waves 4-7 at s_setprio 1 (prio47), pair waves at
# s_setprio 2 (pairprio), edge ring 3 stages ahead (ahead3), InitEdge in 6-wave blocks (init6);
# interleaved, 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
L=deepinteract_amd/lib/variants
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_29_prod_$r.json
  for v in prio47 pairprio ahead3 init6; do
    timeout -k 10 240 python bench.py $B --lib $L/diag_$v/libdeepinteract_amd.so > $O/r6_29_${v}_$r.json
  done
  python tools/show_bench.py $O/r6_29_*_$r.json
done
