#!/bin/bash
# round 6, session 31: rocprofv3 kernel-trace stats (bf16 default, serial, fp32) and FETCH / WRITE
# passes of the final tree (tools/prof_round.sh b)
set -e
bash tools/prof_round.sh b
