#!/bin/bash
# round 6, session 25: the pair stream's launch shape re-swept against the round-6 GeoT kernels
# (persistent edge ring, weight-stationary node layers): blocks x waves 128 x 4 (product) /
# 256 x 2 / 512 x 1 / 64 x 8 / 128 x 3 / 96 x 4, interleaved, 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_25_128x4_$r.json
  for s in 256x2 512x1 64x8 128x3 96x4; do
    timeout -k 10 240 python bench.py $B --pair-blocks ${s%x*} --pair-waves ${s#*x} > $O/r6_25_${s}_$r.json
  done
  python tools/show_bench.py $O/r6_25_*_$r.json
done
