#!/bin/bash
# k_node_fast: XCD-contiguous destination ranges (product) vs launch order (nodelinear)
# node parity, then the overlapped step interleaved (three rounds)
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_nodelinear/libdeepinteract_amd.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
timeout -k 10 200 python tools/diag/dump_forward.py --out $O/g38_prod.pt
timeout -k 10 200 python tools/diag/dump_forward.py --lib $V --out $O/g38_lin.pt
python tools/diag/dump_forward.py --compare $O/g38_prod.pt $O/g38_lin.pt
rm -f $O/g38_*.pt
for r in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub > $O/g38_prod_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --lib $V > $O/g38_lin_$r.json
  python tools/show_bench.py $O/g38_prod_$r.json $O/g38_lin_$r.json
done
