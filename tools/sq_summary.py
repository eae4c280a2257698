"""Aggregate rocprofv3 --pmc counter CSVs (gpurun_out/<dir>/run_counter_collection.csv) into per-kernel
averages per launch, write them to gpurun_out/<out>.csv, and delete the raw per-dispatch directories
(they can exceed gpurun's 64-MiB copy-back limit). usage: sq_summary.py <out> <dir> [<dir> ...]"""
import collections
import csv
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def main(out, dirs):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        path = os.path.join(OUT, d, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        per = collections.defaultdict(float)  # (dispatch, kernel, counter) -> summed value over instances
        for r in csv.DictReader(open(path)):
            per[(r.get("Dispatch_Id", ""), r["Kernel_Name"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, k, c), v in per.items():
            vals[k][c].append(v)
        shutil.rmtree(os.path.join(OUT, d), ignore_errors=True)
    counters = sorted({c for k in vals for c in vals[k]})
    with open(os.path.join(OUT, out + ".csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "launches"] + counters)
        for k in sorted(vals):
            n = max(len(v) for v in vals[k].values())
            w.writerow([k[:120], n] + [f"{sum(vals[k][c]) / len(vals[k][c]):.1f}" if vals[k].get(c) else "" for c in counters])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
