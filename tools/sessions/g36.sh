#!/bin/bash
# k_node_fast: FFN-hidden fragments half prefetched before the first barrier (product) vs all after the O MFMAs (f1late)
# node parity, then the overlapped step interleaved (three rounds)
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_f1late/libdeepinteract_amd.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_node_aggr.py tests/test_gpu_c3.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
timeout -k 10 200 python tools/diag/dump_forward.py --out $O/g36_prod.pt
timeout -k 10 200 python tools/diag/dump_forward.py --lib $V --out $O/g36_late.pt
python tools/diag/dump_forward.py --compare $O/g36_prod.pt $O/g36_late.pt
rm -f $O/g36_*.pt
for r in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub > $O/g36_prod_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --lib $V > $O/g36_late_$r.json
  python tools/show_bench.py $O/g36_prod_$r.json $O/g36_late_$r.json
done
