#!/bin/bash
# Full-size (1024 complexes) bench under the candidate default schedules.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--no-cpu --steps 3 --warmup 1"
tools/gpu_run.sh \
 "f_vec:300:python bench.py $B --pair-kernel vector > gpurun_out/f_vec.json" \
 "f_rows1:300:python bench.py $B --pair-kernel rows --pair-waves 1 > gpurun_out/f_rows1.json" \
 "f_rows2:300:python bench.py $B --pair-kernel rows --pair-waves 2 > gpurun_out/f_rows2.json" \
 "f_rows1_o2:300:python bench.py $B --pair-kernel rows --pair-waves 1 --overlap 2 > gpurun_out/f_rows1_o2.json" \
 "f_vec_mb4:300:python bench.py $B --pair-kernel vector --micro-batch 4 > gpurun_out/f_vec_mb4.json" \
 "f_serial:300:python bench.py $B --overlap 0 > gpurun_out/f_serial.json"
