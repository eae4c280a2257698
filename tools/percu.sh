#!/bin/bash
# Pair-kernel store rate per CU: the row kernel alone on a few CUs (grid = DI_PAIR_BLOCKS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--no-cpu --complexes 64 --steps 2 --warmup 1 --overlap 0"
specs=()
for v in prow_w2 prow_w8 prow_w16; do for nb in 32 64; do
  specs+=("pc_${v}_$nb:200:DI_PAIR_BLOCKS=$nb DI_LIB=$PWD/deepinteract_amd/lib/variants/$v/libdeepinteract_amd.so python bench.py $B > gpurun_out/pc_${v}_$nb.json")
done; done
tools/gpu_run.sh "${specs[@]}"
