#!/bin/bash
# round 6, session 9: which part of InitEdge costs the pair stream its rate (verdict r5 item 3), and
# the pair rate beside the round-6 node layers (tools/diag/interference.py)
set -e
O=gpurun_out; mkdir -p $O
L=deepinteract_amd/lib/variants
timeout -k 10 300 python tools/diag/interference.py > $O/r6_09_interf_product.jsonl
timeout -k 10 200 python tools/diag/interference.py --only init --lib $L/diag_initnopos/libdeepinteract_amd.so > $O/r6_09_interf_initnopos.jsonl
timeout -k 10 200 python tools/diag/interference.py --only init --lib $L/diag_initw0/libdeepinteract_amd.so > $O/r6_09_interf_initw0.jsonl
timeout -k 10 200 python tools/diag/interference.py --only node0,node1 --lib $L/diag_nodefast/libdeepinteract_amd.so > $O/r6_09_interf_nodefast.jsonl
for f in $O/r6_09_interf_*.jsonl; do echo $f; cat $f; done
