#!/bin/bash
# gather record after the bench with the timed schedule released; default bench with sub-records
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py --dist --no-cpu --no-sub --no-prologue --complexes 256 --steps 2 --warmup 1 > $O/g28_dist.json 2>$O/g28_dist.err
python -c "
import json
for l in open('$O/g28_dist.json'):
    if l.startswith('{'): print(json.dumps(json.loads(l)['contact_map_allgather']['predict_sharded']))"
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu > $O/g28_bench.json
python tools/show_bench.py $O/g28_bench.json
python -c "
import json;d=json.load(open('$O/g28_bench.json'));print([ (s.get('what','')[:40], s.get('value')) for s in d['sub_records']])"
