"""Per-kernel average of every counter in rocprofv3 --pmc output directories.

usage: pmc_generic.py OUT.csv LABEL=DIR [LABEL=DIR ...]   (DIR holds run_counter_collection.csv)
Writes one row per (label, kernel, counter): launches and the average value per launch; only the
library's own kernels (di::) are kept."""
import collections
import csv
import os
import sys


def main(out, specs):
    rows = []
    for spec in specs:
        label, d = spec.split("=", 1)
        path = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(path):
            print(f"{label}: no {path}")
            continue
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            if "di::" in r["Kernel_Name"]:
                vals[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in sorted(vals.items()):
            rows.append([label, k[:90], c, len(v), sum(v) / len(v)])
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["label", "kernel", "counter", "launches", "avg_per_launch"])
        w.writerows(rows)
    for r in rows:
        print(f"{r[0]:8s} {r[1][:60]:60s} {r[2]:24s} {r[3]:5d} {r[4]:14.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
