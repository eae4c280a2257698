#!/bin/bash
# round 6, session 1: the RCCL-process collapse of the overlapped schedule (verdict r5 item 1)
# - which stream pairs run concurrently, without and with an RCCL group (queue_probe)
# - the GPU tests that cover the queue (new RCCL-process schedule test, C3 schedule, ragged jobs, ABI)
# - bench.py --dist vs the plain line, interleaved, same box, 1024 complexes per step
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 120 python tools/diag/queue_probe.py > $O/r6_probe_plain.json
timeout -k 10 120 python tools/diag/queue_probe.py --nccl > $O/r6_probe_nccl.json
cat $O/r6_probe_plain.json $O/r6_probe_nccl.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl_schedule.py tests/test_gpu_c3.py tests/test_gpu_parity.py -k "rccl or c3 or pair_queue" -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6_01_pytest.log 2>&1
tail -3 $O/r6_01_pytest.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-sub --no-prologue > $O/r6_01_plain_$r.json
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-sub --no-prologue --dist > $O/r6_01_dist_$r.json
  python tools/show_bench.py $O/r6_01_plain_$r.json $O/r6_01_dist_$r.json
done
