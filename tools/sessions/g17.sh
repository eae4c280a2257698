# round 5 end-of-round profiles (prof_round b) + the gather record with repeated runs
cd $GRAFT_REPO_ROOT
bash tools/prof_round.sh b || exit 1
timeout -k 10 300 python bench.py --dist --no-cpu --no-sub --no-prologue --complexes 256 --steps 2 --warmup 1 > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err
