#!/bin/bash
# CU-partitioned overlap: pair tensor on K dedicated CUs, GeoT on the rest.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--no-cpu --complexes 256 --steps 2 --warmup 1"
tools/gpu_run.sh \
 "cm_tests:300:python -u -m pytest tests/test_gpu_parity.py -k pair -x -q --timeout 120 --timeout-method thread" \
 "cm_base:200:python bench.py $B > gpurun_out/cm_base.json" \
 "cm_s24:200:python bench.py $B --pair-cus 24 > gpurun_out/cm_s24.json" \
 "cm_s32:200:python bench.py $B --pair-cus 32 > gpurun_out/cm_s32.json" \
 "cm_s40:200:python bench.py $B --pair-cus 40 > gpurun_out/cm_s40.json" \
 "cm_s48:200:python bench.py $B --pair-cus 48 > gpurun_out/cm_s48.json" \
 "cm_c32:200:python bench.py $B --pair-cus 32 --cu-layout contig > gpurun_out/cm_c32.json" \
 "cm_s32o2:200:python bench.py $B --pair-cus 32 --overlap 2 > gpurun_out/cm_s32o2.json"
