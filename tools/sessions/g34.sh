#!/bin/bash
# k_node_fast: Q|K|V second-half fragments prefetched before the h exchange (product) vs loaded in
# the Q|K|V loop (qkvjit): node parity, then the overlapped step interleaved
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_qkvjit/libdeepinteract_amd.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_node_aggr.py tests/test_gpu_c3.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
timeout -k 10 200 python tools/diag/dump_forward.py --out $O/g34_prod.pt
timeout -k 10 200 python tools/diag/dump_forward.py --lib $V --out $O/g34_jit.pt
python tools/diag/dump_forward.py --compare $O/g34_prod.pt $O/g34_jit.pt
rm -f $O/g34_*.pt
for r in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub > $O/g34_prod_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --lib $V > $O/g34_jit_$r.json
  python tools/show_bench.py $O/g34_prod_$r.json $O/g34_jit_$r.json
done
