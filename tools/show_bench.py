"""Print value + per-kernel times of bench JSON files."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable:", e)
        continue
    ks = d.get("kernels", {})
    print(f"{f}: {d['value']:.1f} {d['unit'].split()[0]}  {d['ms_per_step']:.1f} ms/step  " +
          "  ".join(f"{k}={v['avg_us']:.0f}" for k, v in ks.items()))
    q = d.get("pair_queue") or {}
    if q:
        print(f"    queue: mode={q.get('mode')} gave_up={q.get('gave_up')} help_fraction={q.get('help_fraction')} "
              f"pair_rate={q.get('pair_rate_GBs')} GB/s")
