#!/bin/bash
# Bench + rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
O="$R/gpurun_out"
mkdir -p "$O"
B="python bench.py"
"$R/tools/gpu_run.sh" \
  "bench:900:$B > $O/bench.json" \
  "prof_stats:900:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --complexes 256" \
  "prof_fetch:900:cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python $R/bench.py --steps 1 --warmup 1 --no-cpu --complexes 64" \
  "prof_write:900:cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python $R/bench.py --steps 1 --warmup 1 --no-cpu --complexes 64"
