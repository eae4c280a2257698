#!/bin/bash
# chunked gather: each round's collective issued at the next put (DI_GATHER_DEFER=1) vs at its own put,
# with 0 / 3 extra streams in the process (3 reproduces the bench context's 5.5-ms exposure)
set -e
for d in 0 1; do
  for n in 0 3; do
    DI_GATHER_DEFER=$d timeout -k 10 200 python tools/diag/gather_probe.py --record --extra-streams $n 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    if 'record_in' in l:
        d=json.loads(l); r=d['record_in_fresh_process']; print('defer=$d extra=$n', {k: r[k] for k in ('compute_only_s','chunked_s','once_s','exposed_collective_s','chunked_equals_once')})"
  done
done
