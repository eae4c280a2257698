#!/bin/bash
# round 6, session 36: end-of-round records after the per-dtype pair-stream default and the
# schedule's resident-InitEdge check: GPU suite, smoke, default / serial / dist / c5 bench lines
# (tools/prof_round.sh a)
set -e
bash tools/prof_round.sh a
