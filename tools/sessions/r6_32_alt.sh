#!/bin/bash
# round 6, session 32: alternative GeoT kernels re-checked at the new pair-stream shape (one 2-wave
# block per CU): InitEdge with LDS-resident weights (--init-kernel split: di_node_embed +
# k_init_res_x32) at its native VGPRs and capped at 160 (diag initres160), the split node layer
# (--node-kernel split: k_node_aggr + k_node_update_ring); interleaved, 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
L=deepinteract_amd/lib/variants
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_32_prod_$r.json
  timeout -k 10 240 python bench.py $B --init-kernel split > $O/r6_32_initres_$r.json
  timeout -k 10 240 python bench.py $B --init-kernel split --lib $L/diag_initres160/libdeepinteract_amd.so > $O/r6_32_initres160_$r.json
  timeout -k 10 240 python bench.py $B --node-kernel split > $O/r6_32_nodesplit_$r.json
  python tools/show_bench.py $O/r6_32_*_$r.json
done
