#!/bin/bash
# Overlapped schedule: edge-kernel variant x pair-tensor launch shape (blocks, kernel), one bench
# run each. usage: SPECS="name:variant:edge_kernel:pair_kernel:pair_blocks[:overlap] ..." tools/pair_sweep.sh
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
V=$R/deepinteract_amd/lib/variants
specs=()
for sp in $SPECS; do
  IFS=: read -r name var ek pk pb ov <<< "$sp"
  specs+=("p_${name}:240:python bench.py --lib $V/$var/libdeepinteract_amd.so --edge-kernel $ek --pair-kernel $pk --pair-blocks $pb --overlap ${ov:-1} --no-cpu --no-prologue --complexes ${CPX:-256} --steps ${STEPS:-3} --warmup 1 > gpurun_out/p_${name}.json")
done
tools/gpu_run.sh "${specs[@]}"
