#!/bin/bash
# InitEdge in 6-wave blocks (init6) vs the product: bit-exactness, then the overlapped step
# interleaved; then bench.py's gather record in a fresh process (vs after the bench run)
set -e
O=gpurun_out; mkdir -p $O
V=deepinteract_amd/lib/variants/diag_init6/libdeepinteract_amd.so
timeout -k 10 200 python tools/diag/dump_forward.py --out $O/g27_prod.pt
timeout -k 10 200 python tools/diag/dump_forward.py --lib $V --out $O/g27_init6.pt
python tools/diag/dump_forward.py --compare $O/g27_prod.pt $O/g27_init6.pt
rm -f $O/g27_*.pt
for r in 1 2; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub > $O/g27_prod_$r.json
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --complexes 512 --no-cpu --no-sub --lib $V > $O/g27_init6_$r.json
  python tools/show_bench.py $O/g27_prod_$r.json $O/g27_init6_$r.json
done
timeout -k 10 300 python tools/diag/gather_probe.py --record > $O/g27_record.jsonl 2>$O/g27_record.err
grep record_in $O/g27_record.jsonl
