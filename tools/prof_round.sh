#!/bin/bash
# One profiling round on the GPU box: GPU parity suite, smoke, bench (default overlapped, serial,
# fp32 supplementary), rocprofv3 kernel-trace stats (bf16 default, serial, fp32), and separate FETCH_SIZE / WRITE_SIZE PMC passes
# for the default (overlapped) and the serial schedules. Outputs under gpurun_out/; summarise with
# tools/pmc_summary.py <tag> and copy the bench lines into profiles/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp; O="$R/gpurun_out"; mkdir -p "$O"
S="--steps 2 --warmup 1 --no-cpu --no-sub --complexes 256"
P="--steps 1 --warmup 1 --no-cpu --no-sub --complexes 64"
F="--dtype f32 --no-prologue --steps 2 --warmup 1 --no-cpu --no-sub --complexes 128"
# usage: tools/prof_round.sh [a|b]   (a: tests + bench lines, b: profiles; default both: one call may
# not hold both within gpurun's limit)
PH="${1:-ab}"
if [[ "$PH" == *a* ]]; then
"$R/tools/gpu_run.sh" \
  "pytest_gpu:600:python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke:200:python __graft_entry__.py smoke" \
  "bench:400:python bench.py --steps 20 --warmup 5 > $O/bench.json" \
  "bench_serial:300:python bench.py --overlap 0 --no-cpu > $O/bench_serial.json" \
  "bench_dist:300:python bench.py --dist --no-cpu --no-sub --no-prologue --complexes 256 --steps 2 --warmup 1 > $O/bench_dist.json" \
  "bench_c5:400:python bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json" \
  || exit $?
fi
if [[ "$PH" == *b* ]]; then
"$R/tools/gpu_run.sh" \
  "fprof_stats:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/fprof_stats -o run -- python3 $R/bench.py $F" \
  "prof_stats:240:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python3 $R/bench.py $S" \
  "prof_fetch:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 $R/bench.py $P" \
  "prof_write:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 $R/bench.py $P" \
  "sprof_stats:240:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/sprof_stats -o run -- python3 $R/bench.py $S --overlap 0" \
  "sprof_fetch:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/sprof_fetch -o run -- python3 $R/bench.py $P --overlap 0" \
  "sprof_write:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/sprof_write -o run -- python3 $R/bench.py $P --overlap 0"
fi
