#!/bin/bash
# Time library variants (tools/build_variants.py) on the GPU: one bench run each, GeoT and the
# pair tensor on one stream so per-kernel times are uncontended.
# usage: tools/variants.sh name1 name2 ...   (BENCH_ARGS to override the bench flags)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
ARGS="${BENCH_ARGS:---no-cpu --overlap 0 --complexes 256 --steps 2 --warmup 1}"
specs=()
for n in "$@"; do
  specs+=("var${TAG}_$n:300:python bench.py --lib $R/deepinteract_amd/lib/variants/$n/libdeepinteract_amd.so $ARGS > gpurun_out/var${TAG}_$n.json")
done
"$R/tools/gpu_run.sh" "${specs[@]}"
