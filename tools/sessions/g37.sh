#!/bin/bash
# edge ring: XCD-contiguous tile order (xcdtiles) vs the product
# node parity, then the overlapped step interleaved (three rounds)
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_xcdtiles/libdeepinteract_amd.so
: timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
timeout -k 10 200 python tools/diag/dump_forward.py --out $O/g37_prod.pt
timeout -k 10 200 python tools/diag/dump_forward.py --lib $V --out $O/g37_xcd.pt
python tools/diag/dump_forward.py --compare $O/g37_prod.pt $O/g37_xcd.pt
rm -f $O/g37_*.pt
for r in 4 5 6; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub > $O/g37_prod_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --lib $V > $O/g37_xcd_$r.json
  python tools/show_bench.py $O/g37_prod_$r.json $O/g37_xcd_$r.json
done
