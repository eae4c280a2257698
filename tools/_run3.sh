#!/bin/bash
# round-3: microbench (+ SQ counters), pair-kernel lines vs rows alone and beside GeoT
R=$PWD; O=$R/gpurun_out; export TMPDIR=/tmp
B="--no-cpu --no-prologue --no-sub --complexes 512 --steps 3 --warmup 1"
tools/gpu_run.sh \
 "sob4:120:./tools/diag/sob_nv4" \
 "sobpmc1:120:cd /tmp && timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/sobpmc1 -o run -- $R/tools/diag/sob_nv4 163840" \
 "sobpmc2:120:cd /tmp && timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/sobpmc2 -o run -- $R/tools/diag/sob_nv4 163840" \
 "p_lines4:150:python bench.py $B --overlap 0 --only pair --pair-kernel lines > $O/p_lines4.json" \
 "p_rows4:150:python bench.py $B --overlap 0 --only pair --pair-kernel rows > $O/p_rows4.json" \
 "p_lines8:150:python bench.py $B --overlap 0 --only pair --pair-kernel lines --pair-waves 8 > $O/p_lines8.json" \
 "p_rows8:150:python bench.py $B --overlap 0 --only pair --pair-kernel rows --pair-waves 8 > $O/p_rows8.json" \
 "o_lines:150:python bench.py $B --pair-kernel lines > $O/o_lines.json" \
 "o_rows:150:python bench.py $B --pair-kernel rows > $O/o_rows.json" \
 "o_lines2:150:python bench.py $B --pair-kernel lines > $O/o_lines2.json" \
 "o_rows2:150:python bench.py $B --pair-kernel rows > $O/o_rows2.json"
