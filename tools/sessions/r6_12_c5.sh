#!/bin/bash
# round 6, session 12: C5 pair-stream grid, second series (session 7: 192 blocks best, 256 x 8 starves GeoT)
set -e
O=gpurun_out; mkdir -p $O
run() { timeout -k 10 240 python bench.py --config c5 --steps 3 --warmup 1 "$@"; }
for r in 1 2; do
  run > $O/r6_12_c5_b128_$r.json
  run --pair-blocks 160 > $O/r6_12_c5_b160_$r.json
  run --pair-blocks 192 > $O/r6_12_c5_b192_$r.json
  run --pair-blocks 224 > $O/r6_12_c5_b224_$r.json
done
python tools/show_bench.py $O/r6_12_c5_*.json
