#!/bin/bash
# micro-batch / pair-grid sweep of the default overlapped schedule (GeoT || vector pair kernel)
B="python bench.py --no-cpu --complexes 256 --steps 2 --warmup 1"
S=()
for mb in 4 16 32; do S+=("mb$mb:120:$B --micro-batch $mb > gpurun_out/mb$mb.json"); done
for pb in 128 192 384 512; do S+=("pb$pb:90:$B --pair-blocks $pb > gpurun_out/pb$pb.json"); done
S+=("ov2:90:$B --overlap 2 > gpurun_out/ov2.json")
tools/gpu_run.sh "${S[@]}"
