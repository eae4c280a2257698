#!/bin/bash
# round 6, session 35: the pair stream's rate beside each GeoT kernel kind at the new default launch
# shape (one 2-wave block per CU; tools/diag/interference.py, as session 9 at 128 x 4)
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/diag/interference.py > $O/r6_35_interf_product.jsonl
cat $O/r6_35_interf_product.jsonl
