"""Summarise variant bench lines (gpurun_out/var*.json): value and per-kernel average µs."""
import glob
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pat = sys.argv[1] if len(sys.argv) > 1 else "var*"
for p in sorted(glob.glob(os.path.join(R, "gpurun_out", pat + ".json"))):
    try:
        d = json.load(open(p))
    except ValueError:
        print(os.path.basename(p), "(no result)")
        continue
    k = d["kernels"]
    print("%-28s %8.1f c/s " % (os.path.basename(p)[:-5], d["value"]),
          " ".join("%s=%.0f" % (n.replace("edge_layer", "el").replace("node_layer", "nl"), r["avg_us"])
                   for n, r in k.items()))
