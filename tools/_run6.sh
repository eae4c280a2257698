#!/bin/bash
# round-3: F kept in registers (keepf variant) vs default, overlapped and serial
R=$PWD; O=$R/gpurun_out; V=$R/deepinteract_amd/lib/variants
B="--no-cpu --no-prologue --no-sub --complexes 512 --steps 3 --warmup 1"
tools/gpu_run.sh \
 "k_base1:120:python bench.py $B > $O/k_base1.json" \
 "k_keep1:120:python bench.py $B --lib $V/keepf/libdeepinteract_amd.so > $O/k_keep1.json" \
 "k_base2:120:python bench.py $B > $O/k_base2.json" \
 "k_keep2:120:python bench.py $B --lib $V/keepf/libdeepinteract_amd.so > $O/k_keep2.json" \
 "k_bases:120:python bench.py $B --overlap 0 > $O/k_bases.json" \
 "k_keeps:120:python bench.py $B --overlap 0 --lib $V/keepf/libdeepinteract_amd.so > $O/k_keeps.json" || exit $?
tools/gpu_run.sh \
 "c_48:120:python bench.py $B --pair-cus 48 > $O/c_48.json" \
 "c_64:120:python bench.py $B --pair-cus 64 > $O/c_64.json" \
 "c_32:120:python bench.py $B --pair-cus 32 > $O/c_32.json" \
 "c_p48:120:python bench.py $B --pair-cus 48 --only pair > $O/c_p48.json" \
 "n_split:120:python bench.py $B --node-kernel split > $O/n_split.json" \
 "n_fused:120:python bench.py $B --node-kernel fused > $O/n_fused.json"
