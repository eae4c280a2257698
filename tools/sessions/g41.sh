#!/bin/bash
# pair-stream grid 128 (default) vs 136 / 144 blocks after the GeoT gains of the end of round 5
set -e
O=gpurun_out; mkdir -p $O
for r in 1 2; do
  for b in 0 136 144; do
    timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --pair-blocks $b > $O/g41_b${b}_$r.json
    python tools/show_bench.py $O/g41_b${b}_$r.json
  done
done
