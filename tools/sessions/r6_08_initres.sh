#!/bin/bash
# round 6, session 8: InitEdge with its weights resident in LDS (zero L2 -> LDS weight stream) capped at
# 160 VGPRs so it co-resides with the pair stream (diag_initres160), as the overlapped InitEdge
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_initres160/libdeepinteract_amd.so
for r in 1 2; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue > $O/r6_08_fused_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue --init-kernel split > $O/r6_08_split168_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue --init-kernel split --lib $V > $O/r6_08_split160_$r.json
  python tools/show_bench.py $O/r6_08_fused_$r.json $O/r6_08_split168_$r.json $O/r6_08_split160_$r.json
done
