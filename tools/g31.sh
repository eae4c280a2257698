#!/bin/bash
# kernel + copy trace of the gather record with 3 extra streams (the 5.5-ms exposure case)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/g31 -o run -- python3 $GRAFT_REPO_ROOT/tools/diag/gather_probe.py --record --extra-streams 3 > $O/g31.out 2>$O/g31.err
grep record_in $O/g31.out
find $O/g31 -name "*.csv" | head
