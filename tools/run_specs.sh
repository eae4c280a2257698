#!/bin/bash
# Run the GPU steps listed in a spec file (one "<name>:<timeout_s>:<command>" per line, default
# tools/_specs.txt) through tools/gpu_run.sh; optional SQ counter passes over a variant library
# (CNT_LIB=<path> CNT_TAG=<tag>). usage on the box: gpurun -- 'bash tools/run_specs.sh [specs]'
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mapfile -t S < "${1:-tools/_specs.txt}"
tools/gpu_run.sh "${S[@]}" || exit $?
[ -n "$CNT_LIB" ] && TAG=$CNT_TAG tools/counters.sh "$CNT_LIB"
exit 0
