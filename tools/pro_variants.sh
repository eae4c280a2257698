#!/bin/bash
# Head-prologue tables-kernel launch-shape variants (lib/variants/pro*, tools: build.build_variant):
# parity tests + rocprofv3 kernel stats of tools/bench_prologue.py per variant, under gpurun_out/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp
steps=()
for v in ${PRO_VARIANTS:-base pro512_cg4 pro1024_cg4 pro512_cg2 pro1024_cg2}; do
  lib="DI_PRO_BASE=1"; [ "$v" != base ] && lib="DI_LIB=$R/deepinteract_amd/lib/variants/$v/libdeepinteract_amd.so"
  steps+=("test_$v:200:$lib python -u -m pytest tests/test_gpu_head_prologue.py -x -q --timeout 120 --timeout-method thread")
  steps+=("stats_$v:200:export $lib; cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/stats_$v -o run -- python $R/tools/bench_prologue.py --reps 5")
done
"$R/tools/gpu_run.sh" "${steps[@]}"
