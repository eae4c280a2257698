#!/bin/bash
# round-3: GPU suite on the pipelined edge kernel, node2 variant, smoke, bench, A/B variants, microbench
V=$PWD/deepinteract_amd/lib/variants
B="--no-cpu --no-prologue --no-sub --complexes 512 --steps 3 --warmup 1"
tools/gpu_run.sh \
 "t_all:900:python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "t_node2:300:DI_TEST_VARIANT=$V/node2/libdeepinteract_amd.so python -u -m pytest tests/test_gpu_node_aggr.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider" \
 "smoke:200:python __graft_entry__.py smoke" \
 "bench:400:python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/b2.json" \
 "v_pipe1_o:200:python bench.py $B > gpurun_out/v_pipe1_o.json" \
 "v_pipe0_o:200:python bench.py $B --lib $V/pipe0/libdeepinteract_amd.so > gpurun_out/v_pipe0_o.json" \
 "v_nv3_o:200:python bench.py $B --lib $V/nv3/libdeepinteract_amd.so > gpurun_out/v_nv3_o.json" \
 "v_nv6_o:200:python bench.py $B --lib $V/nv6/libdeepinteract_amd.so > gpurun_out/v_nv6_o.json" \
 "v_pipe1_s:200:python bench.py $B --overlap 0 > gpurun_out/v_pipe1_s.json" \
 "v_pipe0_s:200:python bench.py $B --overlap 0 --lib $V/pipe0/libdeepinteract_amd.so > gpurun_out/v_pipe0_s.json" \
 "sob:200:for nv in 2 4 6; do ./tools/diag/sob_nv\$nv || exit \$?; done"
