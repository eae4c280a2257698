# round 5: PMC traffic of the persistent pair stream (standalone, every job released), its kernel stats
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_pair_fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/diag/pair_alone.py --stream-only --jobs 4 > $O/pmc_pair_fetch.log 2>&1 || exit 1
timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_pair_write -o run -- python3 $GRAFT_REPO_ROOT/tools/diag/pair_alone.py --stream-only --jobs 4 > $O/pmc_pair_write.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pair_stats -o run -- python3 $GRAFT_REPO_ROOT/tools/diag/pair_alone.py --stream-only --jobs 16 > $O/pair_stats.log 2>&1
