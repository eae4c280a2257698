#!/bin/bash
# round 6, session 11: conflict-free LDS strides in the node kernels (product) vs the first padding
# (diag_ldspad4); node-layer SQ bank-conflict counter; parity
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_ldspad4/libdeepinteract_amd.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_node_aggr.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6_11_pytest.log 2>&1
tail -2 $O/r6_11_pytest.log
for r in 1 2; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue > $O/r6_11_cf_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue --lib $V > $O/r6_11_p4_$r.json
  python tools/show_bench.py $O/r6_11_cf_$r.json $O/r6_11_p4_$r.json
done
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 256 --no-cpu --no-sub --no-prologue --overlap 0 --node-kernel fused > $O/r6_11_cf_serial.json
python tools/show_bench.py $O/r6_11_cf_serial.json
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 110 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/r6_11_pmc -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu --no-prologue --no-sub --complexes 32 --overlap 0 --node-kernel fused > /dev/null 2>&1
python3 $R/tools/sq_summary.py r6_11_sq r6_11_pmc
grep -i node $R/gpurun_out/r6_11_sq.csv
