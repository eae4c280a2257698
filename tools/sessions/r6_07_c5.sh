#!/bin/bash
# round 6, session 7: C5 (2x4000 residues, k=30, 4 layers; pair-bound) pair-stream grid and help cadence
set -e
O=gpurun_out; mkdir -p $O
run() { timeout -k 10 240 python bench.py --config c5 --steps 3 --warmup 1 "$@"; }
for r in 1 2; do
  run > $O/r6_07_c5_default_$r.json
  run --pair-blocks 192 > $O/r6_07_c5_b192_$r.json
  run --pair-blocks 256 > $O/r6_07_c5_b256_$r.json
  run --pair-blocks 256 --pair-waves 8 > $O/r6_07_c5_b256w8_$r.json
  run --help-every 2 > $O/r6_07_c5_he2_$r.json
done
python tools/show_bench.py $O/r6_07_c5_*.json
