#!/bin/bash
# round 6, session 27: the pair stream's default launch shape is now one 2-wave block per CU (was
# 128 x 4): parity of every schedule test, the default bench line (20 steps), the pair stream alone
# at its shapes, C5 shapes (192 x 4 kept so far vs 256 x 2 / 384 x 2 / 256 x 3), then the pair
# stream's standalone FETCH / WRITE passes at the new shape (the line's traffic ratio)
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_rccl_schedule.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6_27_pytest.log 2>&1
tail -2 $O/r6_27_pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > $O/r6_27_bench.json
python tools/show_bench.py $O/r6_27_bench.json
timeout -k 10 200 python tools/diag/pair_alone.py > $O/r6_27_pair_alone.jsonl
cat $O/r6_27_pair_alone.jsonl
C="--config c5 --steps 3 --warmup 1 --no-cpu --no-sub --no-prologue"
for s in 192x4 256x2 384x2 256x3; do
  timeout -k 10 300 python bench.py $C --pair-blocks ${s%x*} --pair-waves ${s#*x} > $O/r6_27_c5_$s.json
done
python tools/show_bench.py $O/r6_27_c5_*.json
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
P="python3 $R/tools/diag/pair_alone.py --stream-only --jobs 4"
timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_pair_fetch -o run -- $P > /dev/null 2>&1
timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_pair_write -o run -- $P > /dev/null 2>&1
ls $O/pmc_pair_fetch $O/pmc_pair_write
