#!/bin/bash
# timing-only variants (results wrong by construction): which part of GeoT the pair stream slows
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
B="python bench.py --no-cpu --no-prologue --complexes 256 --steps 2 --warmup 1"
V="$R/deepinteract_amd/lib/variants"
S=()
for v in base nodma nosilu; do
  S+=("s_$v:120:DI_LIB=$V/$v/libdeepinteract_amd.so $B --overlap 0 > gpurun_out/s_$v.json")
  S+=("o_$v:120:DI_LIB=$V/$v/libdeepinteract_amd.so $B --overlap 1 > gpurun_out/o_$v.json")
done
tools/gpu_run.sh "${S[@]}"
