#!/bin/bash
# hardware-queue aliasing test for the chunked gather's exposure (bench context 5.5 ms vs fresh 0.5 ms)
set -e
O=gpurun_out; mkdir -p $O
for n in 0 3 6; do
  timeout -k 10 200 python tools/diag/gather_probe.py --record --extra-streams $n 2>/dev/null | grep record_in
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --dist --no-cpu --no-sub --no-prologue --complexes 256 --steps 2 --warmup 1 > $O/g29_dist_q8.json 2>$O/g29_dist.err
python -c "
import json
for l in open('$O/g29_dist_q8.json'):
    if l.startswith('{'): d=json.loads(l); print('q8', d['value'], json.dumps(d['contact_map_allgather']['predict_sharded']))"
