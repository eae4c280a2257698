#!/bin/bash
# Edge-layer kernel variants on the GPU (tools/build_variants.py): serial bench timings, then SQ
# counter passes for the default kernel and the lean form. Outputs gpurun_out/v_*.json, pmc*.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=$R/deepinteract_amd/lib/variants
specs=()
for v in ${VARIANTS:-lean4d6 lean4d10 lean12d6 lean8d5}; do
  ek=1; [ "${v#base}" != "$v" ] && ek=0
  for ov in ${OVS:-0}; do
    specs+=("v_${v}_ov${ov}:240:python bench.py --lib $V/$v/libdeepinteract_amd.so --edge-kernel $ek --no-cpu --no-prologue --overlap $ov --complexes 256 --steps 2 --warmup 1 > gpurun_out/v_${v}_ov${ov}.json")
  done
done
tools/gpu_run.sh "${specs[@]}" || exit $?
[ -n "$NO_PMC" ] && exit 0
TAG=_base BENCH_EXTRA="--edge-kernel 0" tools/counters.sh $V/base/libdeepinteract_amd.so || exit $?
TAG=_lean4 BENCH_EXTRA="--edge-kernel 1" tools/counters.sh $V/lean4/libdeepinteract_amd.so
