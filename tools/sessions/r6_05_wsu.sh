#!/bin/bash
# (record: run at the tree where k_node_ws used one chunk of 20 and diag_wsu10 was the two-chunk form;
#  the product now uses chunks of 10 and tools/diag/patch_build.py has the reverse diag, wsu20)
# round 6, session 5: k_node_ws segment sums in one chunk of 20 (product) vs two of 10 (diag_wsu10)
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_wsu10/libdeepinteract_amd.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_node_aggr.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6_05_pytest.log 2>&1
tail -2 $O/r6_05_pytest.log
for r in 1 2; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue > $O/r6_05_u20_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue --lib $V > $O/r6_05_u10_$r.json
  python tools/show_bench.py $O/r6_05_u20_$r.json $O/r6_05_u10_$r.json
done
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 256 --no-cpu --no-sub --no-prologue --overlap 0 --node-kernel fused > $O/r6_05_u20_serial.json
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 256 --no-cpu --no-sub --no-prologue --overlap 0 --node-kernel fused --lib $V > $O/r6_05_u10_serial.json
python tools/show_bench.py $O/r6_05_u20_serial.json $O/r6_05_u10_serial.json
