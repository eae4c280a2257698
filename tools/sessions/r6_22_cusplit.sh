#!/bin/bash
# round 6, session 22: CU-level spatial split of the two dedicated streams (diag cusplit:
# DI_DIAG_GMASK = CUs per XCD taken from GeoT, DI_DIAG_PMASK = CUs per XCD the pair stream runs on,
# 0 = all), vs the product, interleaved, 2 rounds, C3 512 complexes
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_cusplit/libdeepinteract_amd.so
B="--steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --no-prologue"
for r in 1 2; do
  timeout -k 10 240 python bench.py $B > $O/r6_22_prod_$r.json
  for gp in 0_0 4_0 4_4 8_0 8_8 16_16; do
    g=${gp%_*}; p=${gp#*_}
    DI_DIAG_GMASK=$g DI_DIAG_PMASK=$p timeout -k 10 240 python bench.py $B --lib $V > $O/r6_22_g${g}p${p}_$r.json
  done
  python tools/show_bench.py $O/r6_22_*_$r.json
done
