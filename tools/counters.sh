#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, <= 8 SQ counters per pass) over a short serial
# bench; optional first argument: a variant library for bench.py --lib. Outputs gpurun_out/pmc_*.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp; O="$R/gpurun_out"; mkdir -p "$O"
LIB=""; TAG="${TAG:-}"
[ -n "$1" ] && LIB="--lib $(cd "$(dirname "$1")" && pwd)/$(basename "$1")"
B="python3 $R/bench.py $LIB --steps 1 --warmup 1 --no-cpu --no-prologue --complexes 32 --overlap 0 ${BENCH_EXTRA:-}"
"$R/tools/gpu_run.sh" \
  "pmc1${TAG}:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/pmc1${TAG} -o run -- $B" \
  "pmc2${TAG}:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR --output-format csv -d $O/pmc2${TAG} -o run -- $B" \
  "pmc3${TAG}:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/pmc3${TAG} -o run -- $B" && \
python3 "$R/tools/sq_summary.py" "sq${TAG}" "pmc1${TAG}" "pmc2${TAG}" "pmc3${TAG}"
