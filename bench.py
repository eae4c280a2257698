"""Benchmark: complexes/s of the GeoT forward (both chains) + L1xL2 pair tensor.

Workload (BASELINE.json configs[2], the metric's config): synthetic DIPS-Plus-sized heterodimers,
2 x 1000 residues, k = 20, 2 GeoT layers, 128 hidden, 4 heads, bf16 storage / fp32 accumulation;
1024 complexes per GPU per step, processed in micro-batches (a [256,1000,1000] bf16 pair tensor
is 512 MB, so the 1024 outputs cannot be resident at once; each micro-batch's pair tensors are
written to a rotating HBM buffer). The timed region starts with every complex's graph tensors
(node [N,113], edge [E,28], ids) resident in HBM and ends with the outputs in HBM.

Multi-GPU (torchrun): complexes are sharded, each rank owns its 1024; no collective in the timed
region (weak scaling); value = total complexes / max-over-ranks time. After the timed region the
C4 driver (distributed.predict_sharded) runs on real complexes and the contact-map all-gather is
timed at the metric's size (supplementary record).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "complexes/sec GeoT+pair-tensor fwd (2×1k res, k=20, 1/8 GPU); % HBM peak"
METRIC_C5 = "complexes/sec GeoT+pair-tensor fwd (C5 sizing stress: 2×4k res, k=30, 4 GeoT layers)"
HBM_PEAK_GBS = 8000.0
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3}
# SURVEY.md §8d algorithmic MAC per unit (edge or node), per launch kind
EDGE_MAC = {"init_edge": 129_024, "edge_layer": 456_656, "edge_layer_final": 374_736}
H = 128


# MACs the GeoT kernels actually issue on MFMA per edge (packed 16x32 weight blocks x 16 rows per
# 16-edge tile / 16 = 512 MAC per block and edge; the same stage sequence in the bf16 ring kernel and
# fp32 k_edge_layer), by DI_GRAPH_GEO_REF: the reference-equivalent rates above count the
# reference's work (incl. the neighbour-message branch that is exactly zero for reference-featurised
# batches and the nbr_linear the reference applies to 4 gathered rows per edge); these count what runs
EXEC_EDGE_MAC = {True: {"init_edge": 65_536, "edge_layer": 348_160, "edge_layer_final": 266_240},
                 False: {"init_edge": 131_072, "edge_layer": 428_032, "edge_layer_final": 329_728}}
# node kernels issue the node_in_embedding on 128 (113 zero-padded) input columns
EXEC_NODE_EMBED_MAC = 128 * 128 + 3 * 128 * 128


EDGE_KERNEL = {"bf16": "k_edge_x32_ring (v_mfma_f32_32x32x16_bf16, 8-wave weight ring)", "f32": "k_edge_layer (v_mfma_f32_16x16x4_f32)"}


def node_mac(kind):
    q = 3 * H * H
    if kind == "node_embed":
        return 113 * H + q
    if kind == "node_layer":
        return H * H + 2 * H * 2 * H + q
    if kind == "node_layer_final":
        return H * H + 2 * H * 2 * H
    raise KeyError(kind)


def algorithmic_bytes_per_complex(n1, n2, k, s):
    """B = sum_chains [N*113*4 + E*28*4 + E*4 + E*2*nb*4 + N*128*s + E*128*s] + 256*L1*L2*s."""
    b = 0
    for n in (n1, n2):
        e = n * k
        b += n * 113 * 4 + e * 28 * 4 + e * 4 + e * 2 * 2 * 4 + n * 128 * s + e * 128 * s
    return b + 256 * n1 * n2 * s


def algorithmic_flops_per_complex(n1, n2, k, layers=2):
    """2 * sum_chains [E*(129,024 + (L-1)*456,656 + 374,736)
    + N*(113*128 + L*(3*128^2 + 128^2 + 2*128*256))] (77.9 GFLOP at C3)."""
    f = 0
    for n in (n1, n2):
        e = n * k
        f += e * (129_024 + (layers - 1) * 456_656 + 374_736) + n * (113 * H + layers * (3 * H * H + H * H + 2 * H * 2 * H))
    return 2.0 * f


def executed_flops_per_complex(n1, n2, k, layers=2, geo_ref=True):
    """FLOPs the kernels issue on MFMA per complex (EXEC_EDGE_MAC / EXEC_NODE_EMBED_MAC; node layers
    as node_mac): the executed counterpart of algorithmic_flops_per_complex."""
    m = EXEC_EDGE_MAC[bool(geo_ref)]
    f = 0
    for n in (n1, n2):
        e = n * k
        f += e * (m["init_edge"] + (layers - 1) * m["edge_layer"] + m["edge_layer_final"])
        f += n * (EXEC_NODE_EMBED_MAC + (layers - 1) * node_mac("node_layer") + node_mac("node_layer_final"))
    return 2.0 * f


def physical_cores():
    """Physical cores (distinct (package, core) pairs) among the CPUs this process may run on."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    seen = set()
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            with open(base + "physical_package_id") as f1, open(base + "core_id") as f2:
                seen.add((f1.read().strip(), f2.read().strip()))
        except OSError:
            seen.add(("?", str(c)))
    return max(len(seen), 1), len(cpus)


def kernel_units(kind, nodes, edges, l1l2, esz=2):
    """(algorithmic FLOPs, algorithmic HBM bytes) of one launch."""
    if kind == "node_aggr":
        # per in-edge: the gathered V row, its 4 alphas, its source id; per node: in_ptr + the fp32 row out
        return None, edges * (H * esz + 16 + 4) + nodes * (4 + H * 4)
    if kind in EDGE_MAC:
        return 2.0 * EDGE_MAC[kind] * edges, None
    if kind.startswith("node"):
        return 2.0 * node_mac(kind) * nodes, None
    if kind == "pair_tensor":
        return None, l1l2
    raise KeyError(kind)


def dist_setup(force=False):
    """One process per GPU (torchrun env). The RCCL process group is created for WORLD_SIZE > 1, or
    at world size 1 with force (--dist: exercises the collective path on one GPU)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DI_BENCH_REHEARSE=1: every rank on cuda:0 over gloo -- the multi-rank path (barriers, max over
    # ranks, rank-0 line, the gather record) rehearsed on a one-GPU box; RCCL refuses two ranks on
    # one device. Never set for a measurement.
    rehearse = os.environ.get("DI_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    if ws > 1 or force:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        if rehearse:
            dist.init_process_group("gloo", rank=rank, world_size=ws)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=ws, device_id=torch.device("cuda", local))
    return ws, rank, local


def dist_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def barrier(ws):
    if dist_on():
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(ws, x):
    if not dist_on():
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def load_pmc_traffic(kernel, alg_bytes_per_launch=None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (separate
    --pmc passes, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM), or None. The pair stream's
    entry is a ratio to its algorithmic bytes (its launch covers a whole step's jobs, and it is
    profiled standalone: tools/pmc_pair_ratio.py), scaled here to this run's launch."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            rec = json.load(fh).get(kernel, {})
    except (OSError, ValueError):
        return None
    if "hbm_bytes_per_alg_byte" in rec:
        return rec["hbm_bytes_per_alg_byte"] * alg_bytes_per_launch if alg_bytes_per_launch else None
    return rec.get("hbm_bytes_per_launch")


def cpu_baseline(n_res, k, sample, threads, warmup=3):
    """Oracle (CPU restatement, DGL-style op-for-op, fp32, torch.inference_mode) on C3-shaped
    complexes: `warmup` untimed complexes, then `sample` timed (SURVEY.md §8d protocol)."""
    from deepinteract_amd import synth
    from deepinteract_amd.weights import seeded_state_dict
    from oracle import geot_oracle as O
    torch.set_num_threads(threads)
    sd = seeded_state_dict(0, with_head=False)
    ch1, ch2 = synth.synthetic_complex(3, n_res, n_res)
    g1 = O.build_graph(ch1, k=k, seed=1)
    g2 = O.build_graph(ch2, k=k, seed=2)

    def one():
        with torch.inference_mode():
            n1, _ = O.geot_forward(sd, g1)
            n2, _ = O.geot_forward(sd, g2)
            t = O.pair_tensor(n1, n2)
        return t

    for _ in range(warmup):
        one()
    t0 = time.perf_counter()
    for _ in range(sample):
        one()
    dt = time.perf_counter() - t0
    return sample / dt, dt


def head_prologue_record(h1r, h2r, l1, l2, gb, eng, dev, tdt, reps=5):
    """Supplementary, outside the metric: the head's first line
    ELU(inorm_1(conv2d_1(T))) for one micro-batch, fused on HIP from the GeoT node features
    (di_head_prologue; T never materialised). Algorithmic bytes = the [128, L1, L2] output."""
    from deepinteract_amd.engine import HeadPrologueOp
    g = torch.Generator().manual_seed(7)
    C = 128
    w = torch.randn(C, 2 * H, 1, 1, generator=g) / math.sqrt(2 * H)
    op = HeadPrologueOp(w, 0.1 * torch.randn(C, generator=g), 1 + 0.1 * torch.randn(C, generator=g),
                        0.1 * torch.randn(C, generator=g), 1e-6, dev)
    h, _ = eng.forward(gb, clone=False)
    out = torch.empty(sum(C * a * b for a, b in zip(l1, l2)), dtype=tdt, device=dev)
    ev = {}
    op(h, h1r, h2r, l1, l2, out=out)
    torch.cuda.synchronize()
    for _ in range(reps):
        op(h, h1r, h2r, l1, l2, out=out, events=ev)
    torch.cuda.synchronize()
    us = float(np.mean([s.elapsed_time(e) for s, e in ev["head_prologue"]])) * 1e3
    byts = out.numel() * out.element_size()
    return {"op": "ELU(inorm_1(conv2d_1(T))), T never materialised", "complexes": len(l1), "avg_us": round(us, 1),
            "gbs": round(byts / us / 1e3, 1), "frac_hbm": round(byts / us / 1e3 / HBM_PEAK_GBS, 4),
            "bytes_per_launch": byts}


def allgather_record(ws, rank, complexes, n_res, k, dev, reps=3, per_rank=4):
    """Supplementary, outside the metric, two parts:
    1. the C4 driver end to end on REAL maps: distributed.predict_sharded over `per_rank` synthetic
       complexes per rank (device builder -> bf16 GeoT -> pair tensor -> bf16 head -> contact
       probabilities), micro-batches of one complex, timed three ways (after one untimed run each,
       five times interleaved, fastest run kept): no collective (the compute alone), the maps gathered round by round with asynchronous all-gathers overlapped with the
       next micro-batch (chunked, the default) and gathered once at the end; the collectives of the
       chunked plan are then timed alone, giving exposed = t(chunked) - t(compute) and hidden =
       t(collectives alone) - exposed. Every rank checks it holds every map, chunked == once;
    2. one all-gather at the metric's size (`complexes` fp32 [L1, L2] maps per rank), the send
       buffer filled with this rank's real maps (tiled), timed over `reps`."""
    import torch.distributed as dist
    from deepinteract_amd import synth
    from deepinteract_amd.distributed import ChunkedGather, gpu_forward, predict_sharded
    from deepinteract_amd.modules import LitGINI
    from deepinteract_amd.weights import seeded_state_dict
    model = LitGINI(dtype="bf16", head_dtype=torch.bfloat16).to(dev).eval()
    model.load_reference_state_dict(seeded_state_dict(0))
    cx = [synth.synthetic_complex(50_000 + i, n_res, n_res) for i in range(per_rank * ws)]
    fwd = gpu_forward(model, k)
    predict_sharded(cx[:ws], fwd, micro_batch=1, dtype=torch.float32, device=dev, gather="none")  # warm-up

    def run(mode):
        barrier(ws)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        maps, plan = predict_sharded(cx, fwd, micro_batch=1, dtype=torch.float32, device=dev, gather=mode)
        torch.cuda.synchronize()
        return max_over_ranks(ws, time.perf_counter() - t0), maps, plan

    # each mode `reps` times, interleaved, the fastest run of each (one run is ~0.3 s and includes the
    # host-side graph building, whose jitter is larger than the collectives)
    best = {}
    for mode in ("none", "chunked", "once"):  # one untimed run each (the chunked plan's buffers, RCCL setup)
        run(mode)
    for _ in range(max(reps, 5)):
        for mode in ("none", "chunked", "once"):
            t_m, maps_m, plan = run(mode)
            if mode not in best or t_m < best[mode][0]:
                best[mode] = (t_m, maps_m)
    (t_none, mine), (t_chunk, maps), (t_once, maps_once) = best["none"], best["chunked"], best["once"]
    identical = all(torch.equal(a, b) for a, b in zip(maps, maps_once))
    # the chunked plan's collectives alone, on the maps already computed
    sizes = [(n_res, n_res)] * len(cx)
    local = [mine[i] for i in plan[rank]]
    gathers = ChunkedGather(sizes, plan, 1, torch.float32, dev)
    barrier(ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(len(gathers.rounds)):
        ids = gathers.rounds[c][0][rank]
        gathers.put(c, [local[plan[rank].index(i)] for i in ids])
    gathers.finish()
    torch.cuda.synchronize()
    t_coll = max_over_ranks(ws, time.perf_counter() - t0)
    sums = torch.stack([m.double().sum() for m in maps])
    ref = sums.clone()
    dist.broadcast(ref, 0)
    consistent = bool(torch.equal(sums, ref)) and all(0.0 <= float(m.min()) and float(m.max()) <= 1.0 for m in maps)
    exposed = max(t_chunk - t_none, 0.0)
    per_rank_el = complexes * n_res * n_res
    local_flat = torch.cat([m.reshape(-1).float() for m in local])  # the maps as computed (bf16 head) -> fp32 wire
    send = local_flat.repeat((per_rank_el + local_flat.numel() - 1) // local_flat.numel())[:per_rank_el].contiguous()
    recv = torch.empty(per_rank_el * ws, dtype=torch.float32, device=dev)
    dist.all_gather_into_tensor(recv, send)
    torch.cuda.synchronize()
    barrier(ws)
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_gather_into_tensor(recv, send)
    torch.cuda.synchronize()
    dt = max_over_ranks(ws, (time.perf_counter() - t0) / reps)
    del send, recv
    return {"predict_sharded": {"complexes": len(cx), "micro_batch": 1, "rounds": len(gathers.rounds),
                                "compute_only_s": round(t_none, 4), "chunked_s": round(t_chunk, 4),
                                "once_s": round(t_once, 4), "collectives_alone_s": round(t_coll, 4),
                                "exposed_collective_s": round(exposed, 4),
                                "hidden_collective_s": round(max(t_coll - exposed, 0.0), 4),
                                "chunked_equals_once": identical, "maps_consistent_on_all_ranks": consistent,
                                "what": "builder + bf16 GeoT + pair tensor + bf16 head + probs; maps all-gathered "
                                        "per micro-batch round (async, overlapped) vs once at the end"},
            "bytes_per_rank": per_rank_el * 4, "ms": round(dt * 1e3, 3),
            "algbw_GBs": round(per_rank_el * 4 * max(ws - 1, 1) / dt / 1e9, 1),
            "collective": "all_gather_into_tensor (RCCL), real contact maps tiled to the metric's size"}


class SerialSchedule:
    """--overlap 0: GeoT and the pair tensor of each micro-batch one after the other on ONE stream
    (di_pair_tensor, plain stores): the baseline the overlapped schedule is measured against."""

    def __init__(self, eng, pair, mbs, h1r, h2r, l1, l2, pair_buf):
        self.eng, self.pair, self.mbs = eng, pair, mbs
        self.h1r, self.h2r, self.l1, self.l2, self.pair_buf = h1r, h2r, l1, l2, pair_buf

    def step(self, events=None, geot_events=None):
        for gb in self.mbs:
            h, _ = self.eng.forward(gb, clone=False, events=geot_events)
            self.pair(h, self.h1r, self.h2r, self.l1, self.l2, out=self.pair_buf, events=events, hT=self.eng.last_hT)

    def finish(self):
        pass


def timed(sch, steps, warmup, ws=1, kernel_events="dominant"):
    """(elapsed seconds of `steps` steps, bracketed by barrier + synchronize, max over ranks;
    per-kernel HIP event pairs). The overlapped schedule's drain (finish) is inside the timed region.

    kernel_events "dominant" (default): inside the timed region only the pair-tensor launches are
    bracketed by HIP events (the overlapped schedule: ONE pair-stream launch per step), so the dominant
    kernel's roofline is measured live; the GeoT kernels' event pairs come from one untimed step after
    it. "all": every launch in the timed region is bracketed."""
    for _ in range(warmup):
        sch.step()
    sch.finish()
    events = {}
    barrier(ws)
    torch.cuda.synchronize()
    c0 = sch.check() if hasattr(sch, "check") else None
    t0 = time.perf_counter()
    for _ in range(steps):
        sch.step(events, events if kernel_events == "all" else None)
    sch.finish()
    # host time to issue the timed steps (every launch is asynchronous; includes any wait for room in
    # the HIP queues, i.e. back-pressure from the GPU)
    host_issue_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    barrier(ws)
    elapsed = max_over_ranks(ws, time.perf_counter() - t0)
    c1 = sch.check() if hasattr(sch, "check") else None
    if kernel_events != "all":
        sch.step(None, events)
        sch.finish()
        torch.cuda.synchronize()
    # pure host cost of issuing one step, apart from back-pressure: the same step issued onto idle
    # streams (drained first), timed to the end of its issue
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    sch.step()
    host_issue_idle_s = time.perf_counter() - t1
    sch.finish()
    torch.cuda.synchronize()
    queue = None
    if c0 is not None:
        sch.check()
        queue = {"stream_bytes": c1["stream_bytes"] - c0["stream_bytes"], "help_bytes": c1["help_bytes"] - c0["help_bytes"],
                 "gave_up": c1["gave_up"] - c0["gave_up"]}
    return elapsed, events, {"host_issue_s": host_issue_s, "host_issue_idle_s": host_issue_idle_s, "queue": queue,
                             "mode": getattr(sch, "mode", "serial")}


def kernel_table(events, nodes, edges, l1l2, esz, dtype, geo_ref):
    """Per-kernel average duration (HIP events on the launch stream), reference-equivalent TFLOP/s
    (SURVEY §8d MACs), executed TFLOP/s (EXEC_EDGE_MAC) and GB/s of the byte-bound kernels."""
    kern = {}
    for name, pairs in events.items():
        ms = [s.elapsed_time(e) for s, e in pairs]
        avg_s = float(np.mean(ms)) / 1e3
        flops, byts = kernel_units(name, nodes, edges, l1l2, esz)
        rec = {"launches": len(ms), "avg_us": avg_s * 1e6, "total_ms": float(np.sum(ms))}
        if flops is not None:
            rec["tflops"] = flops / avg_s / 1e12
            if name in EXEC_EDGE_MAC[True]:
                rec["exec_tflops"] = 2.0 * EXEC_EDGE_MAC[bool(geo_ref)][name] * edges / avg_s / 1e12
                rec["exec_frac_of_peak"] = rec["exec_tflops"] / MFMA_PEAK_TFLOPS[dtype]
        if byts is not None:
            rec["gbs"] = byts / avg_s / 1e9
        kern[name] = rec
    return kern


def roofline_of(kern, dtype, traffic=None, mfma_only=False):
    """Roofline of the dominant kernel (largest total time; mfma_only: among the GeoT kernels).
    MFMA-bound kernels report executed FLOPs (what the MFMA pipe runs) with the reference-equivalent
    rate beside it."""
    # kernels with a rate only (a pair-stream launch the help launches left no bytes to has none)
    cands = {n: r for n, r in kern.items() if ("tflops" in r if mfma_only else ("tflops" in r or "gbs" in r))}
    dom = max(cands, key=lambda n: cands[n]["total_ms"])
    d = kern[dom]
    if "tflops" in d:
        ach = d.get("exec_tflops", d["tflops"])
        roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_PEAK_TFLOPS[dtype],
                "unit": "TFLOP/s", "flops": "executed" if "exec_tflops" in d else "reference-equivalent",
                "reference_equivalent_tflops": round(d["tflops"], 2)}
    else:
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(d["gbs"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
    roof["traffic"] = traffic
    return roof


def rounded(kern):
    return {n: {kk: round(v, 4) if isinstance(v, float) else v for kk, v in r.items()} for n, r in kern.items()}


def make_schedule(args, eng, mbs, h1r, h2r, l1, l2, tdt, dev, s_geot, s_pair):
    """The timed unit's schedule: overlapped (pair queue beside GeoT, deepinteract_amd.pipeline) or
    serial (--overlap 0)."""
    numel = sum(2 * H * a * b for a, b in zip(l1, l2))
    if args.overlap:
        from deepinteract_amd.pipeline import OverlappedSchedule
        sinks = [torch.empty(numel, dtype=tdt, device=dev) for _ in range(2)]
        # two rotating sinks: the bench never reads the pair tensors back (the parity tests do)
        sch = OverlappedSchedule(eng, mbs, h1r, h2r, l1, l2, sinks, s_geot, s_pair, ring=args.ring,
                                 help_every=args.help_every, stream_blocks=args.pair_blocks,
                                 stream_waves=args.pair_waves, patience_ms=args.patience_ms,
                                 jobs_per_launch=args.jobs_per_launch, discard_outputs=True)
        return sch
    from deepinteract_amd.engine import PairTensorOp
    pair = PairTensorOp(dev, kernel=args.pair_kernel, blocks=args.pair_blocks, waves_per_block=args.pair_waves)
    return SerialSchedule(eng, pair, mbs, h1r, h2r, l1, l2, torch.empty(numel, dtype=tdt, device=dev))


def pair_bytes_per_launch(sch, info, kern, l1l2):
    """Algorithmic bytes of one launch of the dominant (pair-tensor) kernel: the overlapped schedule's
    pair-stream launch covers a step's jobs, of which it writes the bytes the queue counted for it (the
    help launches on the GeoT stream write the rest); the serial kernel writes one micro-batch."""
    if info["queue"] is None:
        return l1l2
    launches = kern.get("pair_tensor", {}).get("launches", 0)
    return info["queue"]["stream_bytes"] / launches if launches else None


def finish_kernel_table(kern, pair_bytes):
    rec = kern.get("pair_tensor")
    if rec is not None:
        if pair_bytes:
            rec["bytes_per_launch"] = pair_bytes
            rec["gbs"] = pair_bytes / (rec["avg_us"] * 1e-6) / 1e9
        else:
            rec.pop("gbs", None)
    return kern


def sub_record(what, dtype, geo_ref, complexes, pool_gb, P, M, n_res, k, args, dev, sd, cfg, s_geot, s_pair,
               steps=3, warmup=1):
    """Supplementary C3 line outside the metric: the same schedule on `complexes` complexes in
    `dtype`, with DI_GRAPH_GEO_REF set or cleared on every batch."""
    from deepinteract_amd.engine import GeoTEngine
    from deepinteract_amd.graph import select_graphs
    eng = GeoTEngine(sd, dtype, cfg, device=dev)
    eng.split_node = args.node_kernel == "split"
    eng.fold_attn = args.node_kernel == "fold"
    eng.fuse_embed_init = args.init_kernel == "fused"
    eng.resident_init = not args.overlap  # beside the pair stream: the staged InitEdge (OverlappedSchedule)
    mbs = [select_graphs(pool_gb, [2 * ((m * M + j) % P) + s for j in range(M) for s in (0, 1)]).with_geo_ref(geo_ref)
           for m in range(complexes // M)]
    gb0 = mbs[0]
    h1r = [gb0.node_off[2 * j] for j in range(M)]
    h2r = [gb0.node_off[2 * j + 1] for j in range(M)]
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    esz = 2 if dtype == "bf16" else 4
    sch = make_schedule(args, eng, mbs, h1r, h2r, [n_res] * M, [n_res] * M, tdt, dev, s_geot, s_pair)
    elapsed, events, info = timed(sch, steps, warmup)
    value = complexes * steps / elapsed
    l1l2 = M * 2 * H * n_res * n_res * esz
    kern = kernel_table(events, gb0.num_nodes, gb0.num_edges, l1l2, esz, dtype, geo_ref)
    kern = finish_kernel_table(kern, pair_bytes_per_launch(sch, info, kern, l1l2))
    flops_c = algorithmic_flops_per_complex(n_res, n_res, k, args.layers)
    xflops_c = executed_flops_per_complex(n_res, n_res, k, args.layers, geo_ref)
    out = {"what": what, "value": round(value, 2), "unit": "complexes/s", "dtype": dtype,
           "geo_ref": bool(geo_ref), "complexes_per_step": complexes, "steps": steps, "warmup": warmup,
           "ms_per_step": round(elapsed / steps * 1e3, 3),
           "mfma_frac_of_peak": round(flops_c * value / (MFMA_PEAK_TFLOPS[dtype] * 1e12), 4),
           "mfma_frac_of_peak_executed": round(xflops_c * value / (MFMA_PEAK_TFLOPS[dtype] * 1e12), 4),
           "hbm_frac_of_peak": round(algorithmic_bytes_per_complex(n_res, n_res, k, esz) * value / (HBM_PEAK_GBS * 1e9), 4),
           "roofline": roofline_of(kern, dtype), "roofline_geot": roofline_of(kern, dtype, mfma_only=True),
           "pair_queue": info["queue"], "kernels": rounded(kern)}
    del mbs, sch, eng
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--complexes", type=int, default=1024, help="complexes per GPU per step")
    ap.add_argument("--micro-batch", type=int, default=8)
    ap.add_argument("--residues", type=int, default=1000)
    ap.add_argument("--knn", type=int, default=20)
    ap.add_argument("--pool", type=int, default=16, help="distinct synthetic complexes replicated in HBM")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--cpu-sample", type=int, default=20)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-prologue", action="store_true", help="skip the supplementary fused-head-prologue line")
    ap.add_argument("--no-sub", action="store_true",
                    help="skip the supplementary fp32 and general-path (geo_ref off) C3 sub-records")
    ap.add_argument("--overlap", type=int, default=1, choices=[0, 1],
                    help="1: GeoT on one stream, the pair tensors on the device-queue pair stream beside it "
                         "(deepinteract_amd.pipeline); 0: both on one stream, one after the other")
    ap.add_argument("--pair-kernel", default="auto", choices=["auto", "lines", "rows", "vector"],
                    help="--overlap 0: the per-micro-batch pair-tensor kernel (auto: row streaming)")
    ap.add_argument("--pair-blocks", type=int, default=0,
                    help="pair-stream blocks (0: one per CU; --overlap 0: resident blocks, 0 = one per CU)")
    ap.add_argument("--pair-waves", type=int, default=0, help="waves per pair block (0: 2 on the pair stream, 4 with --overlap 0)")
    ap.add_argument("--ring", type=int, default=16, help="hT ring slots of the overlapped schedule")
    ap.add_argument("--help-every", type=int, default=4,
                    help="the GeoT stream issues a pair help launch every this many micro-batches")
    ap.add_argument("--jobs-per-launch", type=int, default=0,
                    help="micro-batches per pair-stream launch (0: one launch per step)")
    ap.add_argument("--patience-ms", type=float, default=20.0,
                    help="a pair-stream wave waits at most this long for a micro-batch's signal")
    ap.add_argument("--config", default="c3", choices=["c3", "c5"],
                    help="c3: the metric's workload (BASELINE configs[2]); c5: the 2x4000-residue, k=30, "
                         "4-layer sizing stress (BASELINE configs[4]; no oracle at N > 2304)")
    ap.add_argument("--layers", type=int, default=None, help="GeoT layers (default 2; c5: 4)")
    ap.add_argument("--node-limit", type=int, default=None,
                    help="max_num_graph_nodes of the synthetic model (default 2304; c5: 4096)")
    ap.add_argument("--node-kernel", default=None, choices=["split", "fused", "fold"],
                    help="node layer as di_node_aggregate + di_node_update (split), one di_node_layer (fused), or "
                         "the aggregation folded into the bf16 edge layer + di_node_update_folded (fold). "
                         "Default: fused when overlapped, split otherwise")
    ap.add_argument("--init-kernel", default="fused", choices=["fused", "split"],
                    help="fused: the node embedding as the first blocks of the InitEdge launch (reference-"
                         "featurised batches); split: the embedding, then the resident InitEdge")
    ap.add_argument("--kernel-events", default="dominant", choices=["all", "dominant"],
                    help="HIP events only around the pair-tensor launches in the timed region, the GeoT kernels "
                         "timed in one untimed step after it (dominant, default), or around every launch (all)")
    ap.add_argument("--geo-ref", type=int, default=1, choices=[0, 1],
                    help="0: clear DI_GRAPH_GEO_REF on every batch (the general path; diagnostic)")
    ap.add_argument("--dist", action="store_true",
                    help="create the RCCL process group even at world size 1 (runs the contact-map "
                         "all-gather record on one GPU)")
    ap.add_argument("--lib", default=None, help="a variant build of the HIP library (deepinteract_amd.build."
                                                 "build_variant; tests and diagnostics)")
    args = ap.parse_args()
    if args.lib:
        from deepinteract_amd import _lib
        _lib.load_variant(args.lib)
    if args.config == "c5":
        # BASELINE.json configs[4]: 2x4000 residues, k=30, 4 GeoT layers. The reference's
        # nn.Embedding(max_num_graph_nodes=2304) cannot index 4000 residues, so the synthetic model is
        # built with max_num_graph_nodes=4096 (a LitGINI hyper-parameter); a [256,4000,4000] bf16
        # pair tensor is 8.19 GB, so micro-batches of 2 complexes.
        # the pair stream on 192 blocks x 4 waves (C3: one 2-wave block per CU): C5's GeoT stream is
        # shorter than its pair stream (16.4 GB per micro-batch of 2), so more store waves beside GeoT
        # pay -- round 6, session r6_12: 128 / 160 / 192 / 224 blocks x 4 528 / 551 / 551 / 536
        # complexes/s, pair roofline 0.487 / 0.549 / 0.557 / -- (192: help launches write 1.2 % of the
        # bytes instead of 10 %)
        for key, val in (("residues", 4000), ("knn", 30), ("layers", 4), ("node_limit", 4096), ("pair_blocks", 192),
                         ("pair_waves", 4)):
            if getattr(args, key) in (None, ap.get_default(key)):
                setattr(args, key, val)
        if args.complexes == ap.get_default("complexes"):
            args.complexes = 32
        if args.micro_batch == ap.get_default("micro_batch"):
            args.micro_batch = 2
        args.pool = min(args.pool, 2)
        args.no_cpu = args.no_prologue = args.no_sub = True
    args.layers = args.layers or 2
    args.node_limit = args.node_limit or 2304
    if args.node_kernel is None:
        args.node_kernel = "fused" if args.overlap else "split"
    ws, rank, local = dist_setup(args.dist)
    dev = torch.device("cuda", local)
    from deepinteract_amd import synth
    from deepinteract_amd.builder import build_graph_batch
    from deepinteract_amd.config import GeoTConfig
    from deepinteract_amd.engine import GeoTEngine
    from deepinteract_amd.graph import select_graphs
    from deepinteract_amd.weights import seeded_state_dict

    n_res, k, M = args.residues, args.knn, args.micro_batch
    assert args.complexes % M == 0
    cfg = GeoTConfig(num_gnn_layers=args.layers, knn=k, node_count_limit=args.node_limit)
    sd = seeded_state_dict(0, cfg, with_head=False)
    eng = GeoTEngine(sd, args.dtype, cfg, device=dev)
    eng.split_node = args.node_kernel == "split"
    eng.fold_attn = args.node_kernel == "fold"
    eng.fuse_embed_init = args.init_kernel == "fused"
    eng.resident_init = not args.overlap  # beside the pair stream: the staged InitEdge (OverlappedSchedule)

    # ---- inputs: a pool of distinct complexes built on the device (kNN + features + ids) ----
    P = min(args.pool, args.complexes)
    pool = []
    torch.cuda.synchronize()
    tb = time.perf_counter()
    for c in range(P):
        ch1, ch2 = synth.synthetic_complex(1000 * rank + c, n_res, n_res)
        pool.append((ch1, ch2))
    t_synth = time.perf_counter() - tb
    # the whole pool in one builder call (one launch per stage); neighbour ids as the reference
    # draws them after torch.manual_seed(s) per chain (bit-exact mode). Timed twice: the first
    # (cold) call also pays module loading and the pinned staging allocation.
    t_builds = []
    for _ in range(2):
        torch.cuda.synchronize()
        tb = time.perf_counter()
        pool_gb = build_graph_batch([ch for pair_ in pool for ch in pair_], k=k, device=dev,
                                    node_count_limit=args.node_limit,
                                    nbr_seeds=[2 * (1000 * rank + c) + s + 1 for c in range(P) for s in (0, 1)])
        torch.cuda.synchronize()
        t_builds.append(time.perf_counter() - tb)
    t_build = t_builds[1]
    # resident batch: complexes -> micro-batches (copies of pool complexes, distinct HBM buffers)
    n_mb = args.complexes // M
    mbs = [select_graphs(pool_gb, [2 * ((m * M + j) % P) + s for j in range(M) for s in (0, 1)])
           for m in range(n_mb)]
    if not args.geo_ref:
        mbs = [gb.with_geo_ref(False) for gb in mbs]
    gb0 = mbs[0]
    h1r = [gb0.node_off[2 * j] for j in range(M)]
    h2r = [gb0.node_off[2 * j + 1] for j in range(M)]
    l1 = [n_res] * M
    l2 = [n_res] * M
    tdt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    esz = 2 if args.dtype == "bf16" else 4

    if args.overlap:
        # two streams on hardware queues of their own (deepinteract_amd.pipeline, "Hardware queues"):
        # ordinary streams can share one in a process that holds an RCCL communicator
        from deepinteract_amd.pipeline import schedule_streams
        s_geot, s_pair = schedule_streams(dev)
    else:
        s_geot = s_pair = torch.cuda.current_stream(dev)
    sch = make_schedule(args, eng, mbs, h1r, h2r, l1, l2, tdt, dev, s_geot, s_pair)
    elapsed, events, info = timed(sch, args.steps, args.warmup, ws, args.kernel_events)
    total = args.complexes * args.steps * ws
    value = total / elapsed

    # ---- supplementary (outside the metric) ------------------------------------------------
    prologue = head_prologue_record(h1r, h2r, l1, l2, mbs[-1], eng, dev, tdt) if not args.no_prologue else None
    nodes, edges, geo_ref0 = gb0.num_nodes, gb0.num_edges, gb0.geo_ref
    l1l2 = sum(2 * H * a * b * esz for a, b in zip(l1, l2))
    kern = kernel_table(events, nodes, edges, l1l2, esz, args.dtype, geo_ref0)
    kern = finish_kernel_table(kern, pair_bytes_per_launch(sch, info, kern, l1l2))
    # the gather record runs on its own model and complexes: the timed schedule's buffers (pair
    # sinks, resident micro-batches, engine workspaces) are released first
    del sch, mbs, gb0, eng, events
    gc.collect()
    torch.cuda.empty_cache()
    gather = allgather_record(ws, rank, args.complexes, n_res, k, dev) if dist_on() and args.config == "c3" else None
    # the committed PMC summary was collected on the default workload (C3, micro-batch 8, bf16, the
    # default schedule): any other shape reports traffic null rather than borrowing those bytes
    pmc_shape = (args.config, M, n_res, k, args.layers, args.dtype, args.overlap, args.geo_ref) == \
        ("c3", 8, 1000, 20, 2, "bf16", 1, 1)
    roof = roofline_of(kern, args.dtype)
    if args.overlap and roof["kernel"] == "pair_tensor" and info["mode"] == "overlapped":
        # one persistent launch spans the step: its duration includes the waves' waits for each job's
        # signal, so this is the stream's rate over the step, a lower bound on its store bandwidth
        # (the standalone rate of the same launch shape: tools/diag/pair_alone.py)
        roof["achieved_is"] = "bytes the pair-stream launch stored / its whole duration (waits for signals included)"
    roof["traffic"] = load_pmc_traffic(roof["kernel"], kern.get(roof["kernel"], {}).get("bytes_per_launch")) \
        if pmc_shape else None
    bytes_c = algorithmic_bytes_per_complex(n_res, n_res, k, esz)
    hbm_frac = bytes_c * value / ws / (HBM_PEAK_GBS * 1e9)
    flops_c = algorithmic_flops_per_complex(n_res, n_res, k, args.layers)
    xflops_c = executed_flops_per_complex(n_res, n_res, k, args.layers, geo_ref0)
    mfma_frac = flops_c * value / ws / (MFMA_PEAK_TFLOPS[args.dtype] * 1e12)
    xmfma_frac = xflops_c * value / ws / (MFMA_PEAK_TFLOPS[args.dtype] * 1e12)
    if args.overlap and info["mode"] == "ordered":
        streams = ("ORDERED (the two streams did not run concurrently, di_streams_concurrent): GeoT, then each "
                   "micro-batch's pair tensors by a full-chip help launch on the same stream")
    elif args.overlap:
        streams = (f"GeoT || pair tensor: GeoT on one HIP stream (each micro-batch signalled by the next GeoT launch), the "
                   f"pair tensors on ONE persistent di_pair_stream launch per step on a second stream "
                   f"({args.pair_blocks or ('CUs/2' if args.dtype == 'f32' else 'one per CU')} blocks x "
                   f"{args.pair_waves or (4 if args.dtype == 'f32' else 2)} waves, bounded nt stores, "
                   f"device-queue tickets), di_pair_help on the GeoT stream every {args.help_every} micro-batches "
                   f"(hT ring of {args.ring}) and a drain at the end of the timed steps; no host events between "
                   f"the streams; both streams on hardware queues of their own (CU-masked)")
    else:
        streams = f"1 stream: GeoT then the pair tensor ({args.pair_kernel} kernel) per micro-batch"
    queue = info["queue"]
    if queue is not None:
        tot = queue["stream_bytes"] + queue["help_bytes"]
        queue = dict(queue, mode=info["mode"], help_fraction=round(queue["help_bytes"] / tot, 4) if tot else None,
                     pair_rate_GBs=round(tot / elapsed / 1e9, 1), help_launches_per_step=args.complexes // M // args.help_every)

    out = {
        "metric": METRIC if args.config == "c3" else METRIC_C5, "value": round(value, 2), "unit": "complexes/s", "n_gpus": ws,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (seeded random-walk chains, on-device graph build; seeded random weights)",
        "config": {"workload": f"{args.config.upper()}: 2x{n_res}-residue heterodimers, k={k}, {args.layers} GeoT "
                               f"layers, 128 hidden, 4 heads; "
                               f"GeoT fwd (both chains) + [256,{n_res},{n_res}] pair tensor",
                   "complexes_per_gpu_per_step": args.complexes, "micro_batch": M, "residues": [n_res, n_res],
                   "knn": k, "layers": args.layers, "max_num_graph_nodes": args.node_limit,
                   "parallelism": f"complex-sharded dp{ws}",
                   "streams": streams
                   + ("" if args.geo_ref else "; DI_GRAPH_GEO_REF cleared (general path)")
                   + f"; node layer {args.node_kernel}"
                   + ("; node embedding as the first blocks of the InitEdge launch"
                      if args.init_kernel == "fused" and args.geo_ref else "")
                   + ("; HIP events around every launch in the timed region" if args.kernel_events == "all" else
                      "; HIP events around the pair-tensor launches only (GeoT kernel events from an untimed step)")
                   + f"; edge-layer kernel {EDGE_KERNEL[args.dtype]}"},
        # pure host cost of issuing one step (every launch of the step issued onto drained streams, to
        # the end of its issue): the GPU cannot wait for the host while this stays well below ms_per_step
        "host_issue_ms_per_step": round(info["host_issue_idle_s"] * 1e3, 3),
        # the timed loop's issue time per step; it includes waiting for room in the HIP queues
        # (back-pressure from the GPU), so on a long run it approaches ms_per_step by construction
        "host_issue_timed_region_ms_per_step": round(info["host_issue_s"] / args.steps * 1e3, 3),
        "hbm_frac_of_peak": round(hbm_frac, 4),
        "mfma_frac_of_peak": round(mfma_frac, 4),
        "mfma_frac_of_peak_executed": round(xmfma_frac, 4),
        "algorithmic_per_complex": {"bytes": bytes_c, "flops": flops_c, "executed_mfma_flops": xflops_c,
                                    "mfma_peak_tflops": MFMA_PEAK_TFLOPS[args.dtype], "hbm_peak_gbs": HBM_PEAK_GBS},
        "roofline": roof,
        "roofline_geot": roofline_of(kern, args.dtype, mfma_only=True) if any("tflops" in r for r in kern.values()) else None,
        "pair_queue": queue,
        "kernels": rounded(kern),
        "builder": {"complexes": P, "build_s": round(t_build, 4), "ms_per_complex": round(t_build / P * 1e3, 3),
                    "cold_build_s": round(t_builds[0], 4),
                    "synth_host_s": round(t_synth, 3),
                    "what": "one builder call for the pool: kNN, features, topology, torch-seeded neighbour ids"},
    }
    if prologue is not None:
        out["head_prologue"] = prologue
    if gather is not None:
        out["contact_map_allgather"] = gather
    if not args.no_sub and args.config == "c3":
        # supplementary C3 lines outside the metric (same schedule and kernels): the reference's
        # precision (fp32, deepinteract_utils.py:1088) and the general path with the neighbour-edge
        # gathers live (DI_GRAPH_GEO_REF cleared, deepinteract_modules.py:384-418); the timed
        # schedule's buffers were released above
        out["sub_records"] = [
            sub_record("fp32 C3 (the reference's precision), same schedule", "f32", True, 128, pool_gb, P, M,
                       n_res, k, args, dev, sd, cfg, s_geot, s_pair),
            sub_record("bf16 C3, general path (DI_GRAPH_GEO_REF cleared: neighbour gathers live)", "bf16", False,
                       256, pool_gb, P, M, n_res, k, args, dev, sd, cfg, s_geot, s_pair),
        ]
    if rank == 0 and ws == 1 and not args.no_cpu:
        # the headline at the threads this job is given on the box (OMP_NUM_THREADS: its CPU share),
        # the protocol's one-thread-per-physical-core figure beside it (on a shared host the op-by-op
        # DGL-style path loses to oversubscription there: 0.32 vs 1.19 complexes/s in round 2)
        phys, logical = physical_cores()
        omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
        threads = omp if 0 < omp < phys else phys
        cps, dt = cpu_baseline(n_res, k, args.cpu_sample, threads)
        out["cpu_baseline"] = {"value": round(cps, 4), "unit": "complexes/s", "cores": threads, "kind": "port",
                               "sample": f"{args.cpu_sample} C3 complexes (2x{n_res} res, k={k}) after 3 warm-ups, "
                                         f"oracle fp32 (DGL-style op-for-op) GeoT both chains + pair tensor, "
                                         f"torch.inference_mode, {threads} threads "
                                         + ("(OMP_NUM_THREADS, the job's CPU share)" if threads == omp else
                                            f"= physical cores of the {logical} logical CPUs this process may use")
                                         + f", {dt:.1f}s"}
        if threads != phys:
            cps2, dt2 = cpu_baseline(n_res, k, 5, phys, warmup=1)
            out["cpu_baseline"]["at_physical_cores"] = {"threads": phys, "value": round(cps2, 4),
                                                        "sample": f"5 complexes after 1 warm-up, {dt2:.1f}s"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on():
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
