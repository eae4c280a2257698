#!/bin/bash
# round 6, session 26: the pair stream's launch shape, second series around the winners of session
# 25 (256 x 2 and 512 x 1 beat 128 x 4 by 2 %): 256 x 3 / 768 x 1 / 256 x 4 / 1024 x 1 / 384 x 2,
# interleaved with 128 x 4, 256 x 2, 512 x 1; 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  for s in 128x4 256x2 512x1 256x3 768x1 256x4 1024x1 384x2; do
    timeout -k 10 240 python bench.py $B --pair-blocks ${s%x*} --pair-waves ${s#*x} > $O/r6_26_${s}_$r.json
  done
  python tools/show_bench.py $O/r6_26_*_$r.json
done
