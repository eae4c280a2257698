#!/bin/bash
# is the chunked gather's exposure the persistent edge ring losing CUs to RCCL's blocks?
set -e
V=deepinteract_amd/lib/variants/diag_ring248/libdeepinteract_amd.so
for lib in product ring248; do
  L=""; [ $lib = ring248 ] && L="--lib $V"
  for n in 0 3; do
    timeout -k 10 200 python tools/diag/gather_probe.py --record --extra-streams $n $L 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    if 'record_in' in l:
        d=json.loads(l); r=d['record_in_fresh_process']; print('$lib extra=$n', {k: r[k] for k in ('compute_only_s','chunked_s','once_s','exposed_collective_s')})"
  done
done
