#!/bin/bash
# round 6, session 19: k_node_ws with each tile's residual rows loaded a tile ahead and O's bias held
# for the launch (product) vs the committed tree (rev_head)
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/rev_head/libdeepinteract_amd.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_node_aggr.py tests/test_gpu_c3.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6_19_pytest.log 2>&1
tail -2 $O/r6_19_pytest.log
for r in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue > $O/r6_19_new_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue --lib $V > $O/r6_19_old_$r.json
  python tools/show_bench.py $O/r6_19_new_$r.json $O/r6_19_old_$r.json
done
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 256 --no-cpu --no-sub --no-prologue --overlap 0 --node-kernel fused > $O/r6_19_new_serial.json
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 256 --no-cpu --no-sub --no-prologue --overlap 0 --node-kernel fused --lib $V > $O/r6_19_old_serial.json
python tools/show_bench.py $O/r6_19_new_serial.json $O/r6_19_old_serial.json
