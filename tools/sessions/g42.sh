#!/bin/bash
# fused InitEdge launch: embedding blocks last (product) vs first (embedfirst)
# node parity, then the overlapped step interleaved (three rounds)
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_embedfirst/libdeepinteract_amd.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
timeout -k 10 200 python tools/diag/dump_forward.py --out $O/g42_prod.pt
timeout -k 10 200 python tools/diag/dump_forward.py --lib $V --out $O/g42_ef.pt
python tools/diag/dump_forward.py --compare $O/g42_prod.pt $O/g42_ef.pt
rm -f $O/g42_*.pt
for r in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub > $O/g42_prod_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --lib $V > $O/g42_ef_$r.json
  python tools/show_bench.py $O/g42_prod_$r.json $O/g42_ef_$r.json
done
