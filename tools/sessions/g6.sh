# round 5: full GPU suite, smoke, default bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/g6_pytest.log 2>&1 || exit 1
timeout -k 10 200 python __graft_entry__.py smoke > $O/g6_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/g6_bench.json 2> $O/g6_bench.err
