#!/bin/bash
# gather record with 3 extra streams (the 5.5-ms exposure case): compute on a pool stream instead of
# the null stream; then a kernel + copy trace of the null-stream case
set -e
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for n in 0 3; do
  timeout -k 10 200 python tools/diag/gather_probe.py --record --extra-streams $n --compute-stream 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    if 'record_in' in l:
        d=json.loads(l); r=d['record_in_fresh_process']; print('pool-stream extra=$n', {k: r[k] for k in ('compute_only_s','chunked_s','once_s','exposed_collective_s','chunked_equals_once')})"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/g31 -o run -- python3 $GRAFT_REPO_ROOT/tools/diag/gather_probe.py --record --extra-streams 3 > $O/g31.out 2>$O/g31.err
grep record_in $O/g31.out
find $O/g31 -name "*.csv"
