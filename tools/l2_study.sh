#!/bin/bash
# L2 behaviour of the overlapped vs serial schedule (round 4 study): TCC hit / miss and the EA write
# requests (64-B vs whole) per kernel, each counter pair in its own --pmc pass (<= 4 TCC counters)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp; O="$R/gpurun_out"; mkdir -p "$O"
P="--steps 1 --warmup 1 --no-cpu --no-sub --no-prologue --complexes 64"
specs=("list:60:cd /tmp && rocprofv3 -L > $O/counters_list.txt 2>&1")
for sch in ov ser; do
  X=""; [ "$sch" = ser ] && X="--overlap 0"
  specs+=("hit_$sch:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/hit_$sch -o run -- python3 $R/bench.py $P $X")
  specs+=("wr_$sch:120:cd /tmp && timeout -s KILL 110 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $O/wr_$sch -o run -- python3 $R/bench.py $P $X")
done
"$R/tools/gpu_run.sh" "${specs[@]}"
python3 "$R/tools/pmc_generic.py" "$O/l2_study.csv" hit_ov=$O/hit_ov hit_ser=$O/hit_ser wr_ov=$O/wr_ov wr_ser=$O/wr_ser > "$O/l2_study.txt" 2>&1
rm -rf "$O/hit_ov" "$O/hit_ser" "$O/wr_ov" "$O/wr_ser"
