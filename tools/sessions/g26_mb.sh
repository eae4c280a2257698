#!/bin/bash
# micro-batch 8 / 10 / 12 complexes (1020 complexes per step for 10 and 12; exploratory)
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "8 1024" "10 1020" "12 1020"; do
    set -- $cfg
    timeout -k 10 240 python bench.py --steps 3 --warmup 1 --micro-batch $1 --complexes $2 > gpurun_out/g26_mb$1_$r.json
    python -c "import json;d=json.load(open('gpurun_out/g26_mb$1_$r.json'));print($1,$r,d['value'],d['ms_per_step'])"
  done
done
