#!/bin/bash
# round 6, session 17: end-of-round records (tools/prof_round.sh a: GPU suite, smoke, default /
# serial / dist / c5 bench lines), then the pair stream's standalone PMC ratio
set -e
bash tools/prof_round.sh a
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
P="python3 $R/tools/diag/pair_alone.py --stream-only --jobs 4"
timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_pair_fetch -o run -- $P > /dev/null 2>&1
timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_pair_write -o run -- $P > /dev/null 2>&1
ls $O/pmc_pair_fetch $O/pmc_pair_write
