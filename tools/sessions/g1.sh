cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py::test_pair_queue_ragged_jobs tests/test_gpu_c3.py > gpurun_out/g1_pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --no-sub --no-prologue --complexes 256 --steps 3 --warmup 1 > gpurun_out/g1_bench.json 2> gpurun_out/g1_bench.err && \
timeout -k 10 200 python bench.py --no-cpu --no-sub --no-prologue --complexes 256 --steps 3 --warmup 1 --overlap 0 > gpurun_out/g1_bench_serial.json 2> gpurun_out/g1_bench_serial.err
