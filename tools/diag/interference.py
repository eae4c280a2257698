"""Which GeoT kernel slows the pair stream: the persistent pair stream
(di_pair_stream at the beside shape, every job signalled before the launch) runs over N C3 jobs
while the GeoT stream repeats ONE kernel kind back to back on a C3 micro-batch (its real inputs:
one forward is run first). Per background kind: the pair stream's rate over the window the
background covers, and the background kernel's mean duration beside it, vs both alone.

usage (GPU box): python tools/diag/interference.py [--jobs 12]
One JSON line per background kind (none, init, init_res, edge0, node0, edge1, node1).
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepinteract_amd import _lib, synth  # noqa: E402
from deepinteract_amd.builder import build_graph_batch  # noqa: E402
from deepinteract_amd.engine import GeoTEngine, _ptr  # noqa: E402
from deepinteract_amd.pipeline import PairQueue  # noqa: E402
from deepinteract_amd.weights import seeded_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=12)
    ap.add_argument("--only", default=None, help="comma-separated background kinds")
    ap.add_argument("--lib", default=None, help="a variant / diagnostic build of the library")
    args = ap.parse_args()
    dev = torch.device("cuda")
    lib = _lib.load_variant(args.lib) if args.lib else _lib.load()
    M, L, H = 8, 1000, 128
    eng = GeoTEngine(seeded_state_dict(0, with_head=False), "bf16", device=dev)
    eng.split_node = False
    chains = [c for j in range(M) for c in synth.synthetic_complex(300 + j, L, L)]
    gb = build_graph_batch(chains, k=20, nbr_seeds=list(range(1, 2 * M + 1)), device=dev)
    eng.forward(gb, clone=False)
    torch.cuda.synchronize()
    ws = eng.workspace(gb.num_nodes, gb.num_edges)
    p, g, dt = eng.packed, ctypes.byref(gb.c_graph), _lib.DI_BF16
    h, qkv, f, alpha, hT = ws["h"], ws["qkv"], ws["f"], ws["alpha"], ws["hT"]

    def launch(kind, st):
        if kind == "init":
            rc = lib.di_embed_init_edge(g, dt, gb.node_f.shape[1], _ptr(gb.node_f), _ptr(p.embed[0]), _ptr(p.embed[1]),
                                        _ptr(h[0]), _ptr(qkv[0]), _ptr(gb.edge_f), _ptr(p.init[0]), _ptr(p.init[1]),
                                        _ptr(p.pos_src), _ptr(p.pos_dst), _ptr(f[0]), _ptr(None), -1, st)
        elif kind == "init_res":
            rc = lib.di_init_edge_resident(g, _ptr(gb.edge_f), _ptr(p.init[0]), _ptr(p.init[1]), _ptr(p.pos_src),
                                           _ptr(p.pos_dst), _ptr(f[0]), st)
        elif kind in ("edge0", "edge1"):
            li = 0 if kind == "edge0" else 1
            em, ev = p.edge[li]
            rc = lib.di_edge_layer(g, dt, li, _ptr(gb.edge_f), _ptr(f[li]), _ptr(None), _ptr(qkv[li]), _ptr(em),
                                   _ptr(ev), _ptr(alpha), _ptr(None if li else f[1]), _ptr(None), st)
        else:
            li = 0 if kind == "node0" else 1
            nm, nv = p.node[li]
            rc = lib.di_node_layer(g, dt, li, _ptr(alpha), _ptr(h[li]), _ptr(qkv[li]), _ptr(nm), _ptr(nv),
                                   _ptr(h[1 - li]), _ptr(None if li else qkv[1]), _ptr(hT if li else None), st)
        _lib.check(rc, kind)

    # pair jobs: C3 micro-batches reading this batch's hT
    n_rows = gb.num_nodes
    descs = (_lib.DiPairDesc * M)()
    off = 0
    for i in range(M):
        descs[i] = _lib.DiPairDesc(gb.node_off[2 * i], gb.node_off[2 * i + 1], off, L, L)
        off += 2 * H * L * L
    d_descs = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    sinks = [torch.empty(off, dtype=torch.bfloat16, device=dev) for _ in range(2)]
    items = lib.di_pair_job_items(M, L, H)
    q = PairQueue(dev, args.jobs)
    q.set_jobs([_lib.DiPairJob(hT.data_ptr(), d_descs.data_ptr(), sinks[j % 2].data_ptr(), n_rows, M, L, items)
                for j in range(args.jobs)])
    launch_cfg = _lib.DiPairLaunch(_lib.DI_PAIR_ROWS, 0, 0, 1)
    from deepinteract_amd.pipeline import schedule_streams
    s_geot, s_pair = schedule_streams(dev)  # hardware queues of their own
    job_bytes = 2 * off

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def alone(kind, n=20):
        with torch.cuda.stream(s_geot):
            launch(kind, ctypes.c_void_p(s_geot.cuda_stream))
            a, b = ev(), ev()
            a.record()
            for _ in range(n):
                launch(kind, ctypes.c_void_p(s_geot.cuda_stream))
            b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / n

    def beside(kind, reps_per_job):
        q.reset()
        torch.cuda.synchronize()
        with torch.cuda.stream(s_pair):
            stp = ctypes.c_void_p(s_pair.cuda_stream)
            _lib.check(lib.di_pair_signal(ctypes.c_void_p(q.state.data_ptr()), args.jobs - 1, stp), "signal")
            pa, pb = ev(), ev()
            pa.record()
            _lib.check(lib.di_pair_stream(dt, ctypes.c_void_p(q.jobs.data_ptr()), 0, args.jobs, H,
                                          ctypes.c_void_p(q.state.data_ptr()), ctypes.byref(launch_cfg), 20.0, stp),
                       "stream")
            pb.record()
        n = 0
        if kind != "none":
            with torch.cuda.stream(s_geot):
                stg = ctypes.c_void_p(s_geot.cuda_stream)
                ga, gb_ = ev(), ev()
                ga.record()
                n = max(1, int(reps_per_job * args.jobs))
                for _ in range(n):
                    launch(kind, stg)
                gb_.record()
        torch.cuda.synchronize()
        t_pair = pa.elapsed_time(pb) * 1e3
        rec = {"background": kind, "pair_us_per_job": t_pair / args.jobs,
               "pair_tb_s": job_bytes * args.jobs / (t_pair * 1e-6) / 1e12}
        if n:
            t_g = ga.elapsed_time(gb_) * 1e3
            rec.update({"launches": n, "kernel_us_beside": t_g / n, "kernel_us_alone": alone(kind),
                        "window_frac_of_pair": t_g / t_pair})
            if base["rate"] and t_g < t_pair:
                # the pair bytes written while the background ran, if the rest of the window ran at the
                # unloaded rate (both launches start together)
                b_bg = job_bytes * args.jobs - (t_pair - t_g) * 1e-6 * base["rate"] * 1e12
                rec["pair_tb_s_during_background"] = b_bg / (t_g * 1e-6) / 1e12
        return rec

    base = {"rate": None}
    r0 = beside("none", 0)
    base["rate"] = r0["pair_tb_s"]
    print(json.dumps(r0))
    # enough launches to cover ~80 % of the pair window (pair ~1 ms per job beside)
    kinds = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else \
        ["init", "init_res", "edge0", "node0", "edge1", "node1"]
    est = {"init": 140, "init_res": 140, "edge0": 430, "node0": 52, "edge1": 330, "node1": 45}
    for kind in kinds:
        us = est[kind]
        print(json.dumps(beside(kind, 800.0 / us)), flush=True)


if __name__ == "__main__":
    main()
