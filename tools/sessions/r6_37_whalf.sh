#!/bin/bash
# round 6, session 37: how much of the edge layers' cost to the pair stream is their L2 -> LDS weight
# stream: the ring's stages DMA'd at half their blocks (diag whalf, timing only) vs the product; pair
# rate beside the edge layers (tools/diag/interference.py) and the step (2 interleaved rounds)
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_whalf/libdeepinteract_amd.so
timeout -k 10 200 python tools/diag/interference.py --only edge0,edge1 > $O/r6_37_interf_product.jsonl
timeout -k 10 200 python tools/diag/interference.py --only edge0,edge1 --lib $V > $O/r6_37_interf_whalf.jsonl
cat $O/r6_37_interf_*.jsonl
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_37_prod_$r.json
  timeout -k 10 240 python bench.py $B --lib $V > $O/r6_37_whalf_$r.json
  python tools/show_bench.py $O/r6_37_*_$r.json
done
