#!/bin/bash
# edge ring: XCD-contiguous tiles in both layers (product) vs the final layer only (xcdfinal)
# node parity, then the overlapped step interleaved (three rounds)
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_xcdfinal/libdeepinteract_amd.so
: timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
timeout -k 10 200 python tools/diag/dump_forward.py --out $O/g40_prod.pt
timeout -k 10 200 python tools/diag/dump_forward.py --lib $V --out $O/g40_xf.pt
python tools/diag/dump_forward.py --compare $O/g40_prod.pt $O/g40_xf.pt
rm -f $O/g40_*.pt
for r in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub > $O/g40_prod_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --lib $V > $O/g40_xf_$r.json
  python tools/show_bench.py $O/g40_prod_$r.json $O/g40_xf_$r.json
done
