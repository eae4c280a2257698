# round 5: in-kernel signal; GPU parity of the touched paths, bench A/B, kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
B="--no-cpu --no-sub --no-prologue --complexes 512 --steps 3 --warmup 1"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c3.py tests/test_gpu_parity.py tests/test_gpu_node_aggr.py tests/test_gpu_api.py > $O/g4_pytest.log 2>&1 && \
timeout -k 10 150 python bench.py $B > $O/g4_a1.json 2>/dev/null && \
timeout -k 10 150 python bench.py $B > $O/g4_a2.json 2>/dev/null && \
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/g4_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-sub --no-prologue --complexes 256 --steps 2 --warmup 1 > $O/g4_trace.json 2>/dev/null)
