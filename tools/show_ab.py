"""Summarise bench JSON lines: value, ms/step, pair-queue counters, roofline and GeoT kernel times.
usage: python tools/show_ab.py gpurun_out/<prefix>*.json"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.load(open(f))
    except (OSError, ValueError) as e:
        print(f, "unreadable", e)
        continue
    q = d.get("pair_queue") or {}
    k = d["kernels"]
    print(f"{f.split('/')[-1]:28s} {d['value']:8.1f} {d['ms_per_step']:8.2f} ms  help {q.get('help_fraction')} "
          f"gave_up {q.get('gave_up')} pair {q.get('pair_rate_GBs')} GB/s  roof {d['roofline']['achieved']}  "
          + " ".join(f"{n[:10]}={v['avg_us']:.0f}" for n, v in k.items() if n != "pair_tensor"))
