#!/bin/bash
# round 6, session 32: alternative GeoT launches re-checked at the new pair-stream shape (one 2-wave
# block per CU): the node embedding as its own launch before the staged InitEdge (--init-kernel
# split; the LDS-resident InitEdge cannot share a SIMD with a store wave and the schedule now refuses
# it: its first run here had every pair wave give up), the split node layer (--node-kernel split:
# k_node_aggr + k_node_update_ring); interleaved, 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_32_prod_$r.json
  timeout -k 10 240 python bench.py $B --init-kernel split > $O/r6_32_initsplit_$r.json
  timeout -k 10 240 python bench.py $B --node-kernel split > $O/r6_32_nodesplit_$r.json
  python tools/show_bench.py $O/r6_32_*_$r.json
done
