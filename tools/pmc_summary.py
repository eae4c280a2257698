"""Summarise a profiling round (tools/prof_round.sh output under gpurun_out/) into profiles/.

* profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied verbatim)
* profiles/<tag>_pmc.csv            per-kernel average FETCH_SIZE / WRITE_SIZE (KiB per launch)
* profiles/pmc_traffic.json         HBM bytes per launch per bench kernel name, read by bench.py

HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE counts 64 B per 128-B read request
on gfx950 and reads 1/2 of a wide coalesced stream (MI355X_MICROARCH.md §HBM); WRITE_SIZE is exact
for 16-B-per-lane stores. The doubling is calibrated for 16-B/lane streams only; narrower gathers
are uncalibrated (stated next to the numbers).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {
    "k_node_embed": "node_embed", "k_init_edge": "init_edge", "k_edge_layer<di::F32T, 0": "edge_layer",
    "k_edge_layer<di::F32T, 1": "edge_layer_final", "k_node_layer<di::BF16T, false>": "node_layer",
    "k_node_layer<di::BF16T, true>": "node_layer_final",
    "k_edge_lean<0": "edge_layer", "k_edge_lean<1": "edge_layer_final", "k_node_aggr<di::BF16T>": "node_aggr",
    "k_edge_x32_ring<0": "edge_layer", "k_edge_x32_ring<1": "edge_layer_final", "k_init_x32": "init_edge",
    "k_init_res_x32": "init_edge",
    "k_node_ws<false>": "node_layer", "k_node_ws<true>": "node_layer_final",
    "k_node_fast<false": "node_layer", "k_node_fast<true": "node_layer_final",
    "k_node_update_ring<false>": "node_layer", "k_node_update_ring<true>": "node_layer_final", "k_pair_lines": "pair_tensor", "k_pair_rows": "pair_tensor", "k_pair_vec": "pair_tensor",
    "k_pair_flat": "pair_tensor", "k_pair_stream": "pair_tensor", "k_pair_help": "pair_help",
    "k_prologue_rows": "head_prologue_rows", "k_prologue_tables": "head_prologue_tables",
    "k_knn": "knn", "k_geo_feats": "geo_feats", "k_geo_stats": "geo_stats", "k_nbr_ids": "nbr_ids",
}


def bench_name(kernel):
    for key, name in NAMES.items():
        if key in kernel:
            return name
    return None


def main(tag, src=os.path.join(ROOT, "gpurun_out"), prefix="prof", traffic_json=True):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(src, f"{prefix}_stats", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    agg = collections.defaultdict(dict)
    for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(os.path.join(src, f"{prefix}_{kind}", "run_counter_collection.csv"))):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            agg[k][counter] = sum(v) / len(v)
    traffic = {}
    with open(os.path.join(prof, f"{tag}_pmc.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "FETCH_SIZE_KiB_per_launch", "WRITE_SIZE_KiB_per_launch", "hbm_bytes_per_launch"])
        for k, d in sorted(agg.items()):
            f, wr = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0)
            hbm = (2 * f + wr) * 1024
            w.writerow([k, f"{f:.1f}", f"{wr:.1f}", f"{hbm:.0f}"])
            name = bench_name(k)
            if name:
                traffic[name] = {"hbm_bytes_per_launch": hbm, "fetch_kib": f, "write_kib": wr, "source": f"{tag}_pmc.csv"}
    if traffic_json:
        # the pair stream's standalone ratio (tools/pmc_pair_ratio.py) is kept over this run's
        # figure for it: rocprofv3 --pmc serialises the overlapped schedule's dispatches
        path = os.path.join(prof, "pmc_traffic.json")
        if os.path.exists(path):
            for k, v in json.load(open(path)).items():
                if "hbm_bytes_per_alg_byte" in v:
                    traffic[k] = v
        with open(path, "w") as fh:
            json.dump(traffic, fh, indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    # usage: pmc_summary.py <tag> [<prefix> [--no-traffic-json]]
    a = sys.argv[1:]
    main(a[0] if a else "r1", prefix=a[1] if len(a) > 1 else "prof", traffic_json="--no-traffic-json" not in a)
