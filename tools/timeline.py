"""Stream occupancy and kernel-boundary gaps of the overlapped C3 schedule from a rocprofv3 kernel
trace (kernel timeline).

usage: python tools/timeline.py <run_kernel_trace.csv | profiles/<tag>_timeline.csv> [--save out.csv]

Collect the trace on the GPU box with
  cd /tmp && rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace -o run \\
      -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu --no-sub --no-prologue --complexes 256
Prints, over the steady-state window (the middle 60 % of the traced span of the final node layers):
the micro-batch period, each stream's busy fraction (pair stream: the persistent k_pair_stream
launches, or the per-micro-batch pair kernels of older schedules; GeoT stream: every other kernel,
help and signal launches included), the time the GeoT stream spends in pair help launches, the
GeoT stream's boundary gap by (preceding, next) kernel and the mean kernel durations."""
import collections
import csv
import sys

KINDS = [("k_pair_stream", "pstream"), ("k_pair_help", "help"), ("k_pair_signal", "signal"),
         ("k_pair_rows", "pair"), ("k_pair_lines", "pair"), ("k_pair_vec", "pair"),
         ("k_edge_layer<di::F32T, 0", "edge0"), ("k_edge_layer<di::F32T, 1", "edge1"),
         ("k_init_edge", "init"), ("k_node_layer<di::BF16T, false", "node0"), ("k_node_layer<di::BF16T, true", "node1"),
         ("k_node_layer<di::F32T, false", "node0"), ("k_node_layer<di::F32T, true", "node1"),
         ("k_node_aggr", "aggr"), ("k_node_update_ring<false", "node0"), ("k_node_update_ring<true", "node1"),
         ("k_node_embed", "embed"), ("k_edge_x32_ring<0", "edge0"), ("k_edge_x32_ring<1", "edge1"), ("k_init_x32", "init"),
         ("k_init_res_x32", "init")]
PAIR_STREAM = ("pstream", "pair")


def kind(name):
    for key, k in KINDS:
        if key in name:
            return k
    return None


def load(path):
    rows = list(csv.DictReader(open(path)))
    if rows and "Start_Timestamp" in rows[0]:  # raw rocprofv3 trace (ns)
        return [(int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3, r["Kernel_Name"])
                for r in rows if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    return [(float(r["start_us"]), float(r["end_us"]), r["kernel"]) for r in rows]  # profiles/ copy (µs)


def union(xs, t0, t1):
    """Length of the union of intervals clipped to [t0, t1]."""
    iv = sorted((max(s, t0), min(e, t1)) for s, e, *_ in xs if e > t0 and s < t1)
    tot, cur_s, cur_e = 0.0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(argv):
    ev = sorted((s, e, kind(n), n) for s, e, n in load(argv[0]) if kind(n))
    if "--save" in argv:
        t0 = ev[0][0]
        with open(argv[argv.index("--save") + 1], "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["kernel", "stream", "start_us", "end_us"])
            for s, e, k, n in ev:
                w.writerow([n[:80], "pair" if k in PAIR_STREAM else "geot", round(s - t0, 2), round(e - t0, 2)])
    ends = [x for x in ev if x[2] == "node1"]
    if len(ends) < 10:
        raise SystemExit("need a trace with at least 10 micro-batches")
    a, b = int(len(ends) * 0.2), int(len(ends) * 0.8)
    t0, t1 = ends[a][1], ends[b][1]
    span, nmb = t1 - t0, b - a
    pair = [x for x in ev if x[2] in PAIR_STREAM]
    geot = [x for x in ev if x[2] not in PAIR_STREAM]
    print(f"window {span / 1e3:.2f} ms, {nmb} micro-batches, period {span / nmb:.1f} us")
    print(f"pair stream busy {union(pair, t0, t1) / span:.3f}")
    gb = union(geot, t0, t1)
    help_t = union([x for x in geot if x[2] == "help"], t0, t1)
    print(f"GeoT stream busy {gb / span:.3f} (help launches {help_t / span:.3f} of the window, "
          f"{help_t / nmb:.1f} us per micro-batch); idle {(span - gb) / nmb:.1f} us per micro-batch")
    gw = [x for x in geot if x[0] >= t0 and x[1] <= t1]
    gaps = collections.defaultdict(list)
    for p, q in zip(gw, gw[1:]):
        gaps[(p[2], q[2])].append(q[0] - p[1])
    for k, v in sorted(gaps.items()):
        print(f"  gap {k[0]:>6} -> {k[1]:<6} n={len(v):4d} mean {sum(v) / len(v):7.1f} us")
    dur = collections.defaultdict(list)
    for s, e, k, _ in ev:
        if s >= t0 and e <= t1:
            dur[k].append(e - s)
    print("  mean durations (us):", {k: round(sum(v) / len(v), 1) for k, v in dur.items()})
    print("  launches in window:", {k: len(v) for k, v in dur.items()})


if __name__ == "__main__":
    main(sys.argv[1:])
