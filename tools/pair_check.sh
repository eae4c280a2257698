#!/bin/bash
# Pair-tensor parity tests, then isolated / overlapped timing at a few grid sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--no-cpu --complexes 256 --steps 2 --warmup 1"
tools/gpu_run.sh \
 "pair_tests:300:python -u -m pytest tests/test_gpu_parity.py -k pair -x -q --timeout 120 --timeout-method thread" \
 "p_serial:200:python bench.py $B --overlap 0 > gpurun_out/p_serial.json" \
 "p_ov:200:python bench.py $B > gpurun_out/p_ov.json" \
 "p_ov512:200:DI_PAIR_BLOCKS=512 python bench.py $B > gpurun_out/p_ov512.json" \
 "p_ov128:200:DI_PAIR_BLOCKS=128 python bench.py $B > gpurun_out/p_ov128.json" \
 "p_serial512:200:DI_PAIR_BLOCKS=512 python bench.py $B --overlap 0 > gpurun_out/p_serial512.json"
