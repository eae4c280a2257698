#!/bin/bash
# Interleaved A/B of bench configurations on one box: tools/ab.sh ROUNDS "name|bench args" ...
# (C3, 512 complexes, 3 steps; variant libraries via --lib). Outputs gpurun_out/ab_<name><round>.json;
# summarise with tools/show_bench.py gpurun_out/ab_*.json
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"; O="$R/gpurun_out"; mkdir -p "$O"
B="--no-cpu --no-prologue --no-sub --complexes 512 --steps 3 --warmup 1"
N=$1; shift
specs=()
for i in $(seq 1 "$N"); do
  for c in "$@"; do
    name="${c%%|*}"; args="${c#*|}"
    specs+=("ab_$name$i:150:python bench.py $B $args > $O/ab_$name$i.json")
  done
done
tools/gpu_run.sh "${specs[@]}"
