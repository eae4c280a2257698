#!/bin/bash
# round 6, session 6: the pair stream ALONE on 1/2/3/4/6 of the 8 XCDs (verdict r5 item 4): blocks on
# the other XCDs exit at once (tools/diag/patch_build.py pairxcdN); full-chip product for reference
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 120 python tools/diag/pair_alone.py --jobs 8 --shapes 128x4,256x4,256x8 > $O/r6_06_xcd8.jsonl
for n in 1 2 3 4 6; do
  timeout -k 10 120 python tools/diag/pair_alone.py --jobs 8 --shapes 256x4,256x8,256x16 --lib deepinteract_amd/lib/variants/diag_pairxcd$n/libdeepinteract_amd.so > $O/r6_06_xcd$n.jsonl
done
for f in $O/r6_06_xcd*.jsonl; do echo $f; cat $f; done
