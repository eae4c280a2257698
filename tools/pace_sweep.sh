B="python bench.py --no-cpu --complexes 256 --steps 2 --warmup 1"
S=()
for p in 0 1 2 4 8; do S+=("vec$p:90:$B --pair-kernel vector --pair-pace $p > gpurun_out/vec$p.json"); done
for p in 0 4 8 16 32; do S+=("rows$p:90:$B --pair-kernel rows --pair-pace $p > gpurun_out/rows$p.json"); done
tools/gpu_run.sh "${S[@]}"
