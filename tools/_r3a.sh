#!/bin/bash
# round 3: GPU suite, smoke, default bench line; A/B of the span pair kernel, resident InitEdge,
# embed side stream, keep-F (overlapped and serial)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"; O="$R/gpurun_out"; mkdir -p "$O"
V=$R/deepinteract_amd/lib/variants
B="--no-cpu --no-prologue --no-sub --complexes 512 --steps 3 --warmup 1"
A="--no-cpu --no-prologue --no-sub --complexes 256 --steps 3 --warmup 1 --only pair --pair-beside 0 --pair-waves 4"
tools/gpu_run.sh \
  "t_new:300:python -u -m pytest tests/test_gpu_parity.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider -k 'pair_tensor or init_edge_resident or geot_matches'" \
  "ab_base1:120:python bench.py $B > $O/ab_base1.json" \
  "ab_stg1:120:python bench.py $B --lib $V/initstaged/libdeepinteract_amd.so > $O/ab_stg1.json" \
  "ab_r16:120:python bench.py $B --lib $V/initres16/libdeepinteract_amd.so > $O/ab_r16.json" \
  "ab_noemb:120:python bench.py $B --embed-stream 0 > $O/ab_noemb.json" \
  "ab_span1:120:python bench.py $B --pair-kernel span > $O/ab_span1.json" \
  "ab_keepf:120:python bench.py $B --lib $V/keepf/libdeepinteract_amd.so > $O/ab_keepf.json" \
  "ab_base2:120:python bench.py $B > $O/ab_base2.json" \
  "ab_stg2:120:python bench.py $B --lib $V/initstaged/libdeepinteract_amd.so > $O/ab_stg2.json" \
  "ab_span2:120:python bench.py $B --pair-kernel span > $O/ab_span2.json" \
  "se_base:120:python bench.py $B --overlap 0 > $O/se_base.json" \
  "se_stg:120:python bench.py $B --overlap 0 --lib $V/initstaged/libdeepinteract_amd.so > $O/se_stg.json" \
  "al_span:120:python bench.py $A --pair-kernel span > $O/al_span.json" \
  "al_rows:120:python bench.py $A --pair-kernel rows > $O/al_rows.json"
