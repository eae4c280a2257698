cd $GRAFT_REPO_ROOT
B="--no-cpu --complexes 256 --steps 2 --warmup 1"
tools/gpu_run.sh \
 "pb64:200:DI_PAIR_BLOCKS=64 python bench.py $B > gpurun_out/k_pb64.json" \
 "pb128:200:DI_PAIR_BLOCKS=128 python bench.py $B > gpurun_out/k_pb128.json" \
 "pb512:200:DI_PAIR_BLOCKS=512 python bench.py $B > gpurun_out/k_pb512.json" \
 "pb1024:200:DI_PAIR_BLOCKS=1024 python bench.py $B > gpurun_out/k_pb1024.json" \
 "mb4:200:python bench.py $B --micro-batch 4 > gpurun_out/k_mb4.json" \
 "mb16:200:python bench.py $B --micro-batch 16 > gpurun_out/k_mb16.json" \
 "mb32:200:python bench.py $B --micro-batch 32 > gpurun_out/k_mb32.json"
