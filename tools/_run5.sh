#!/bin/bash
# round-3: VALU issue microbench, GPU suite, node2 variant, packed vs scalar f32 VALU A/B
R=$PWD; O=$R/gpurun_out; V=$R/deepinteract_amd/lib/variants
B="--no-cpu --no-prologue --no-sub --complexes 512 --steps 3 --warmup 1"
tools/gpu_run.sh \
 "vib:60:tools/diag/vib > $O/vib.txt" \
 "t_all:600:python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "t_node2:200:DI_TEST_VARIANT=$V/node2/libdeepinteract_amd.so python -u -m pytest tests/test_gpu_node_aggr.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider" \
 "v_base1:120:python bench.py $B > $O/v_base1.json" \
 "v_scal1:120:python bench.py $B --lib $V/scalar/libdeepinteract_amd.so > $O/v_scal1.json" \
 "v_nosl1:120:python bench.py $B --lib $V/noslp/libdeepinteract_amd.so > $O/v_nosl1.json" \
 "v_base2:120:python bench.py $B > $O/v_base2.json" \
 "v_scal2:120:python bench.py $B --lib $V/scalar/libdeepinteract_amd.so > $O/v_scal2.json" \
 "v_bases:120:python bench.py $B --overlap 0 > $O/v_bases.json" \
 "v_scals:120:python bench.py $B --overlap 0 --lib $V/scalar/libdeepinteract_amd.so > $O/v_scals.json"
