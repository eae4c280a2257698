#!/bin/bash
# parity (fast fail) + short rocprofv3 kernel-trace stats of the bench
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp; O="$R/gpurun_out"; mkdir -p "$O"
"$R/tools/gpu_run.sh" \
  "pytest_gpu:600:python -m pytest tests/test_gpu_parity.py -q -m gpu -rf -x" \
  "prof_stats:900:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --complexes 256 ${BENCH_ARGS}" \
  "bench:900:python bench.py --no-cpu ${BENCH_ARGS} > $O/bench.json"
