#!/bin/bash
# A/B of the XCD-aware edge-tile order: GPU parity first, then serial (per-kernel) and overlapped
# benches of the base (XCD-aware) and noxcd variants.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
B="python bench.py --no-cpu --no-prologue --complexes 256 --steps 2 --warmup 1"
V="$R/deepinteract_amd/lib/variants"
tools/gpu_run.sh \
  "pytest_gpu:400:python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "s_base:120:DI_LIB=$V/base/libdeepinteract_amd.so $B --overlap 0 > gpurun_out/s_base.json" \
  "s_noxcd:120:DI_LIB=$V/noxcd/libdeepinteract_amd.so $B --overlap 0 > gpurun_out/s_noxcd.json" \
  "o_base:120:DI_LIB=$V/base/libdeepinteract_amd.so $B > gpurun_out/o_base.json" \
  "o_noxcd:120:DI_LIB=$V/noxcd/libdeepinteract_amd.so $B > gpurun_out/o_noxcd.json" \
  "o_base2:120:DI_LIB=$V/base/libdeepinteract_amd.so $B > gpurun_out/o_base2.json" \
  "o_noxcd2:120:DI_LIB=$V/noxcd/libdeepinteract_amd.so $B > gpurun_out/o_noxcd2.json"
