#!/bin/bash
# round-3: GPU suite, node2 variant, split vs fused node layer beside the pair stream
R=$PWD; O=$R/gpurun_out; V=$R/deepinteract_amd/lib/variants
B="--no-cpu --no-prologue --no-sub --complexes 512 --steps 3 --warmup 1"
tools/gpu_run.sh \
 "t_all:900:python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "t_node2:300:DI_TEST_VARIANT=$V/node2/libdeepinteract_amd.so python -u -m pytest tests/test_gpu_node_aggr.py -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider" \
 "n_fused1:150:python bench.py $B --node-kernel fused > $O/n_fused1.json" \
 "n_split1:150:python bench.py $B --node-kernel split > $O/n_split1.json" \
 "n_fused2:150:python bench.py $B --node-kernel fused > $O/n_fused2.json" \
 "n_split2:150:python bench.py $B --node-kernel split > $O/n_split2.json" \
 "n_ser:150:python bench.py $B --overlap 0 > $O/n_ser.json" \
 "n_ser_fused:150:python bench.py $B --overlap 0 --node-kernel fused > $O/n_ser_fused.json"
