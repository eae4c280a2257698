#!/bin/bash
# round 6, session 34: the fp32 schedule (the reference's precision) at the new pair-stream default
# shape (256 x 2) vs round 5's 128 x 4; interleaved, 2 rounds, 128 complexes
set -e
O=gpurun_out; mkdir -p $O
B="--dtype f32 --steps 3 --warmup 1 --complexes 128 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_34_f32_256x2_$r.json
  timeout -k 10 240 python bench.py $B --pair-blocks 128 --pair-waves 4 > $O/r6_34_f32_128x4_$r.json
  python tools/show_bench.py $O/r6_34_*_$r.json
done
