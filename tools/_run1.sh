#!/bin/bash
# round-3 validation: GPU suite, node2 variant, smoke, bench, SiLU-overlap microbenchmark
tools/gpu_run.sh \
 "t_all:900:python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "t_node2:300:DI_TEST_VARIANT=$PWD/deepinteract_amd/lib/variants/node2/libdeepinteract_amd.so python -u -m pytest tests/test_gpu_node_aggr.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider" \
 "smoke:200:python __graft_entry__.py smoke" \
 "bench:400:python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/b1.json" \
 "sob:200:for nv in 2 4 6; do ./tools/diag/sob_nv\$nv || exit \$?; done"
