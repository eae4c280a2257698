#!/bin/bash
# round 6, session 30: end-of-round records of the final tree (pair stream one 2-wave block per CU):
# GPU suite, smoke, default / serial / dist / c5 bench lines (tools/prof_round.sh a)
set -e
bash tools/prof_round.sh a
