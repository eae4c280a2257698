#!/bin/bash
# pair tensor after InitEdge (overlap 2) with the row-streaming kernel, pacing sweep
B="python bench.py --no-cpu --no-prologue --complexes 256 --steps 2 --warmup 1"
S=()
for p in 0 2 4 8; do S+=("ov2rows$p:120:$B --overlap 2 --pair-kernel rows --pair-pace $p > gpurun_out/ov2rows$p.json"); done
S+=("ov2vec:120:$B --overlap 2 --pair-kernel vector > gpurun_out/ov2vec.json")
S+=("ov1vec:120:$B --overlap 1 --pair-kernel vector > gpurun_out/ov1vec.json")
tools/gpu_run.sh "${S[@]}"
