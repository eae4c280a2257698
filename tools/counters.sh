#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp; O="$R/gpurun_out"; mkdir -p "$O"
B="python $R/bench.py --steps 1 --warmup 1 --no-cpu --complexes 32 --overlap 0"
"$R/tools/gpu_run.sh" \
  "list:300:cd /tmp && rocprofv3 -L > $O/counters_list.txt 2>&1" \
  "bench_noov:900:python bench.py --no-cpu --overlap 0 > $O/bench_noov.json" \
  "pmc_sq1:900:cd /tmp && rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/pmc_sq1 -o run -- $B" \
  "pmc_sq2:900:cd /tmp && rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM --output-format csv -d $O/pmc_sq2 -o run -- $B" \
  "pmc_sq3:900:cd /tmp && rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq3 -o run -- $B"
