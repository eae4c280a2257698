#!/bin/bash
# micro-batch 8 vs 16 on the current kernels (interleaved, two rounds)
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for mb in 8 16; do
    timeout -k 10 240 python bench.py --steps 3 --warmup 1 --micro-batch $mb > gpurun_out/g25_mb${mb}_$r.json
    python -c "import json,sys;d=json.load(open('gpurun_out/g25_mb${mb}_$r.json'));print($mb,$r,d['value'],d['ms_per_step'])"
  done
done
