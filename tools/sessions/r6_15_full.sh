#!/bin/bash
# round 6, session 15: full GPU suite + smoke on the current tree; default bench (the driver's
# command) and --dist at 1024 complexes (verdict r5 item 1: within 3 %)
set -e
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6_15_pytest.log 2>&1 || { tail -30 $O/r6_15_pytest.log; exit 1; }
tail -3 $O/r6_15_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/r6_15_smoke.log 2>&1
tail -2 $O/r6_15_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --no-sub --no-prologue > $O/r6_15_plain.json
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --no-sub --no-prologue --dist > $O/r6_15_dist.json
python tools/show_bench.py $O/r6_15_plain.json $O/r6_15_dist.json
