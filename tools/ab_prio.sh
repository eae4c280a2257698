#!/bin/bash
# GeoT wave priority / persistent edge tiles beside the pair-tensor store stream
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
B="python bench.py --no-cpu --no-prologue --complexes 256 --steps 2 --warmup 1"
V="$R/deepinteract_amd/lib/variants"
S=()
for v in base prio1 prio3 pp_persist persist_prio2; do
  S+=("ov1vec_$v:120:DI_LIB=$V/$v/libdeepinteract_amd.so $B --overlap 1 --pair-kernel vector > gpurun_out/ov1vec_$v.json")
  S+=("ov1rows_$v:120:DI_LIB=$V/$v/libdeepinteract_amd.so $B --overlap 1 --pair-kernel rows > gpurun_out/ov1rows_$v.json")
  S+=("ov2rows_$v:120:DI_LIB=$V/$v/libdeepinteract_amd.so $B --overlap 2 --pair-kernel rows > gpurun_out/ov2rows_$v.json")
done
tools/gpu_run.sh "${S[@]}"
