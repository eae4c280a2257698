#!/bin/bash
# rehearsal of bench.py's multi-rank path on a one-GPU box: 2 ranks on cuda:0 over gloo
set -e
O=gpurun_out; mkdir -p $O
DI_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 2 --warmup 1 --complexes 64 --no-cpu --no-sub > $O/g39_ws2.json 2> $O/g39_ws2.err
python -c "
import json
for l in open('$O/g39_ws2.json'):
    if l.startswith('{'):
        d=json.loads(l); print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], json.dumps(d.get('contact_map_allgather',{}).get('predict_sharded')))"
