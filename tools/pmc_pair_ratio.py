"""HBM traffic of the persistent pair stream per algorithmic byte, from separate rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE passes over `tools/diag/pair_alone.py --stream-only --jobs J` (every job
released before the launch: under --pmc the profiler serialises dispatches, so the stream cannot run
beside GeoT there and the bench's own PMC pass sees only help launches). Writes the ratio into
profiles/pmc_traffic.json["pair_tensor"]; bench.py scales it by the bytes of the metric run's stream
launch (roofline.traffic).

usage: python tools/pmc_pair_ratio.py <tag> <jobs_per_launch> [<src dir prefix, default pmc_pair>]
HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md §HBM gfx950 correction)."""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JOB_BYTES = 8 * 2 * 128 * 1000 * 1000 * 2  # one C3 micro-batch of pair tensors (bf16)


def main(tag, jobs, prefix="pmc_pair"):
    src = os.path.join(ROOT, "gpurun_out")
    sums, disp = {}, {}
    for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        path = os.path.join(src, f"{prefix}_{kind}", "run_counter_collection.csv")
        rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter and "k_pair_stream" in r["Kernel_Name"]]
        sums[counter] = sum(float(r["Counter_Value"]) for r in rows)
        disp[counter] = len({r.get("Dispatch_Id", i) for i, r in enumerate(rows)})
        shutil.copy(path, os.path.join(ROOT, "profiles", f"{tag}_pmc_pair_{kind}.csv"))
    launches = disp["WRITE_SIZE"]
    alg = launches * jobs * JOB_BYTES
    hbm = (2 * sums["FETCH_SIZE"] + sums["WRITE_SIZE"]) * 1024
    rec = {"hbm_bytes_per_alg_byte": hbm / alg, "launches": launches, "jobs_per_launch": jobs,
           "fetch_kib_per_job": sums["FETCH_SIZE"] / (launches * jobs),
           "write_kib_per_job": sums["WRITE_SIZE"] / (launches * jobs),
           "source": f"{tag}_pmc_pair_fetch.csv / _write.csv (tools/diag/pair_alone.py --stream-only)"}
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    d = json.load(open(path)) if os.path.exists(path) else {}
    d["pair_tensor"] = rec
    with open(path, "w") as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[1]), a[2] if len(a) > 2 else "pmc_pair")
