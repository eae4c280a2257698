#!/bin/bash
# round 6, session 24: the committed tree after the A/B sessions 20-23 (product sources unchanged
# since 1397ab2): GPU suite, smoke, default / serial / dist / c5 bench lines (tools/prof_round.sh a)
set -e
bash tools/prof_round.sh a
