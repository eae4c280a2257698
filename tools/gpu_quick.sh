#!/bin/bash
# Quick GPU check: the split node layer / x32 edge tests, then a serial and an overlapped bench.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tools/gpu_run.sh \
 "t_aggr:300:python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_node_aggr.py tests/test_gpu_edge_x32.py" \
 "b_ser:240:python bench.py --no-cpu --no-prologue --overlap 0 --complexes 256 --steps 2 --warmup 1 > gpurun_out/b_ser.json" \
 "b_ov:240:python bench.py --no-cpu --no-prologue --complexes 256 --steps 4 --warmup 1 > gpurun_out/b_ov.json" || exit $?
exit 0
