#!/bin/bash
# round 3: interleaved A/B (3 rounds): resident InitEdge (+ index prefetch) vs the staged kernel,
# node embedding on the side stream vs the main stream, node layer in the 4-slot ring vs double-buffered
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"; O="$R/gpurun_out"; mkdir -p "$O"
V=$R/deepinteract_amd/lib/variants
B="--no-cpu --no-prologue --no-sub --complexes 512 --steps 3 --warmup 1"
T="-q -rf --timeout 150 --timeout-method thread -p no:cacheprovider"
specs=("t_init:200:python -u -m pytest tests/test_gpu_parity.py $T -k 'init_edge_resident or geot_matches'"
       "t_node:200:python -u -m pytest tests/test_gpu_node_aggr.py $T")
for i in 1 2 3; do
  specs+=("b_base$i:120:python bench.py $B > $O/b_base$i.json")
  specs+=("b_noemb$i:120:python bench.py $B --embed-stream 0 > $O/b_noemb$i.json")
  specs+=("b_stg$i:120:python bench.py $B --lib $V/initstaged/libdeepinteract_amd.so > $O/b_stg$i.json")
  specs+=("b_ndb$i:120:python bench.py $B --lib $V/nodedbuf/libdeepinteract_amd.so > $O/b_ndb$i.json")
done
specs+=("b_nopf:120:python bench.py $B --lib $V/initnopf/libdeepinteract_amd.so > $O/b_nopf.json")
specs+=("s_base:120:python bench.py $B --overlap 0 > $O/s_base.json")
specs+=("s_nopf:120:python bench.py $B --overlap 0 --lib $V/initnopf/libdeepinteract_amd.so > $O/s_nopf.json")
specs+=("s_fused:120:python bench.py $B --overlap 0 --node-kernel fused > $O/s_fused.json")
tools/gpu_run.sh "${specs[@]}"
