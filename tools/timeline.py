"""Stream occupancy and kernel-boundary gaps of the overlapped C3 schedule from a rocprofv3 kernel
trace ("Where the overlapped step's time goes").

usage: python tools/timeline.py <run_kernel_trace.csv | profiles/r3_v2_timeline.csv> [--save out.csv]

Collect the trace on the GPU box with
  cd /tmp && rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace -o run \\
      -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu --no-sub --no-prologue --complexes 256
Prints, over the steady-state window (the pair launches after the first 40 % of the run): each
stream's busy fraction, the pair stream's idle time per micro-batch, the GeoT stream's boundary gap
by (preceding, next) kernel, and the average kernel durations."""
import collections
import csv
import sys

KINDS = [("k_pair_rows", "pair"), ("k_pair_lines", "pair"), ("k_pair_vec", "pair"), ("k_edge_lean<0", "edge0"),
         ("k_edge_lean<1", "edge1"), ("k_edge_layer<di::F32T, 0", "edge0"), ("k_edge_layer<di::F32T, 1", "edge1"),
         ("k_init_edge", "init"), ("k_node_layer<di::BF16T, false", "node0"), ("k_node_layer<di::BF16T, true", "node1"),
         ("k_node_layer<di::F32T, false", "node0"), ("k_node_layer<di::F32T, true", "node1"),
         ("k_node_aggr", "aggr"), ("k_node_update_ring<false", "node0"), ("k_node_update_ring<true", "node1"),
         ("k_node_embed", "embed"), ("k_edge_x32<0", "edge0"), ("k_edge_x32<1", "edge1"), ("k_init_x32", "init"),
         ("k_init_res_x32", "init")]


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


def main(argv):
    ev = sorted((s, e, kind(n), n) for s, e, n in load(argv[0]) if kind(n))
    if "--save" in argv:
        t0 = ev[0][0]
        with open(argv[argv.index("--save") + 1], "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["kernel", "stream", "start_us", "end_us"])
            for s, e, _, n in ev:
                w.writerow([n[:80], "", round(s - t0, 2), round(e - t0, 2)])
    pairs = [x for x in ev if x[2] == "pair"]
    if len(pairs) < 10:
        raise SystemExit("need an overlapped trace with at least 10 pair-tensor launches")
    win = pairs[int(len(pairs) * 0.4):-2]
    t0, t1 = win[0][0], win[-1][1]
    span = t1 - t0

    def busy(xs):
        return sum(min(e, t1) - max(s, t0) for s, e, *_ in xs if e > t0 and s < t1) / span

    geot = [x for x in ev if x[2] not in ("pair", "embed") and x[0] >= t0 and x[1] <= t1]
    print(f"window {span / 1e3:.2f} ms, {len(win)} micro-batches, period {span / len(win):.1f} us")
    print(f"pair stream busy {busy(pairs):.3f}; idle {(1 - busy(pairs)) * span / len(win):.1f} us per micro-batch")
    print(f"GeoT stream busy {busy(geot):.3f}")
    gaps = collections.defaultdict(list)
    for a, b in zip(geot, geot[1:]):
        gaps[(a[2], b[2])].append(b[0] - a[1])
    for k, v in sorted(gaps.items()):
        print(f"  gap {k[0]:>6} -> {k[1]:<6} n={len(v):3d} mean {sum(v) / len(v):6.1f} us")
    dur = collections.defaultdict(list)
    for s, e, k, _ in ev:
        if s >= t0 and e <= t1:
            dur[k].append(e - s)
    print("  mean durations (us):", {k: round(sum(v) / len(v), 1) for k, v in dur.items()})


if __name__ == "__main__":
    main(sys.argv[1:])
