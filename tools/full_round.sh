#!/bin/bash
# GPU parity suite, then bench + rocprofv3 kernel-trace stats + separate PMC passes.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp; O="$R/gpurun_out"; mkdir -p "$O"
"$R/tools/gpu_run.sh" \
  "pytest_gpu:420:python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "bench:300:python bench.py ${BENCH_ARGS} > $O/bench.json" \
  "prof_stats:240:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --complexes 256 ${BENCH_ARGS}" \
  "prof_fetch:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python $R/bench.py --steps 1 --warmup 1 --no-cpu --complexes 64 ${BENCH_ARGS}" \
  "prof_write:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python $R/bench.py --steps 1 --warmup 1 --no-cpu --complexes 64 ${BENCH_ARGS}"
