#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
B="python bench.py --no-cpu --no-prologue --complexes 256 --steps 2 --warmup 1 --overlap 0"
V="$R/deepinteract_amd/lib/variants"
tools/gpu_run.sh "s_base:120:DI_LIB=$V/base/libdeepinteract_amd.so $B > gpurun_out/s_base.json" \
  "s_nw8:120:DI_LIB=$V/nw8/libdeepinteract_amd.so $B > gpurun_out/s_nw8.json" \
  "s_mb4:120:$B --micro-batch 4 > gpurun_out/s_mb4.json" \
  "s_mb16:120:$B --micro-batch 16 > gpurun_out/s_mb16.json"
