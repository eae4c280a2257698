#!/bin/bash
# round-3: pipelined-epilogue A/B (interleaved repeats), overlapped and serial
R=$PWD; O=$R/gpurun_out; V=$R/deepinteract_amd/lib/variants
B="--no-cpu --no-prologue --no-sub --complexes 512 --steps 3 --warmup 1"
specs=()
for rep in 1 2; do
  for v in main pipe0 nv2 nv3 nv5; do
    L=""; [ $v != main ] && L="--lib $V/$v/libdeepinteract_amd.so"
    specs+=("ab_${v}_o$rep:150:python bench.py $B $L > $O/ab_${v}_o$rep.json")
  done
done
for v in main pipe0 nv3; do
  L=""; [ $v != main ] && L="--lib $V/$v/libdeepinteract_amd.so"
  specs+=("ab_${v}_s:150:python bench.py $B --overlap 0 $L > $O/ab_${v}_s.json")
done
tools/gpu_run.sh "${specs[@]}"
