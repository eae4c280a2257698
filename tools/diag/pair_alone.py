"""The pair-tensor stream ALONE (no GeoT beside it), at the beside launch shapes: how much of the
beside-GeoT rate (~3.95 TB/s per micro-batch job) is the stream's own ceiling and how much is
interference.

usage (GPU box): python tools/diag/pair_alone.py [--jobs 16]
Prints one JSON line per configuration: the persistent stream (di_pair_stream, every job signalled
before the launch) at several grids, the full-chip help launch (di_pair_help) and the one-shot kernel
(di_pair_tensor rows, plain stores), each over the same C3 jobs (8 complexes of 1000 x 1000).
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepinteract_amd import _lib  # noqa: E402
from deepinteract_amd.pipeline import PairQueue  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=16)
    ap.add_argument("--complexes", type=int, default=8)
    ap.add_argument("--res", type=int, default=1000)
    ap.add_argument("--shapes", default=None,
                    help="only di_pair_stream at these grids, e.g. '256x4,256x8' (XCD-restricted variants)")
    ap.add_argument("--stream-only", action="store_true",
                    help="only the beside shape (128 x 4 stream): the PMC traffic pass (tools/pmc_pair_ratio.py)")
    ap.add_argument("--lib", default=None, help="a variant / diagnostic build of the library")
    args = ap.parse_args()
    if args.lib:
        _lib.load_variant(args.lib)
    lib, dev = _lib.load(), torch.device("cuda")
    H, M, L = 128, args.complexes, args.res
    n_rows = 2 * M * L
    hT = [torch.randn(H, n_rows, device=dev).bfloat16() for _ in range(2)]
    descs = (_lib.DiPairDesc * M)()
    off = 0
    for i in range(M):
        descs[i] = _lib.DiPairDesc(2 * i * L, (2 * i + 1) * L, off, L, L)
        off += 2 * H * L * L
    d_descs = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    sinks = [torch.empty(off, dtype=torch.bfloat16, device=dev) for _ in range(2)]
    job_bytes = off * 2
    items = lib.di_pair_job_items(M, L, H)
    s = torch.cuda.current_stream()
    st = ctypes.c_void_p(s.cuda_stream)

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            t = a.elapsed_time(b) / 1e3
            best = t if best is None else min(best, t)
        return best

    def queue_run(kind, blocks, waves):
        q = PairQueue(dev, args.jobs)
        jobs = [_lib.DiPairJob(hT[j % 2].data_ptr(), d_descs.data_ptr(), sinks[j % 2].data_ptr(), n_rows, M, L, items)
                for j in range(args.jobs)]
        q.set_jobs(jobs)
        launch = _lib.DiPairLaunch(_lib.DI_PAIR_ROWS, blocks, waves, 1 if kind == "stream" else 0)

        def fn():
            q.reset()
            _lib.check(lib.di_pair_signal(ctypes.c_void_p(q.state.data_ptr()), args.jobs - 1, st), "signal")
            if kind == "stream":
                _lib.check(lib.di_pair_stream(_lib.DI_BF16, ctypes.c_void_p(q.jobs.data_ptr()), 0, args.jobs, H,
                                              ctypes.c_void_p(q.state.data_ptr()), ctypes.byref(launch), 20.0, st),
                           "stream")
            else:
                _lib.check(lib.di_pair_help(_lib.DI_BF16, ctypes.c_void_p(q.jobs.data_ptr()), 0, args.jobs - 1, H,
                                            ctypes.c_void_p(q.state.data_ptr()), ctypes.byref(launch), -1, st), "help")
        t = timed(fn)
        c = q.counters()
        return t, c

    out = []
    if args.shapes:
        for shape in args.shapes.split(","):
            blocks, waves = (int(x) for x in shape.split("x"))
            t, c = queue_run("stream", blocks, waves)
            print(json.dumps({"what": "di_pair_stream (bounded nt stores)", "blocks": blocks, "waves": waves,
                              "us_per_job": 1e6 * t / args.jobs, "tb_s": job_bytes * args.jobs / t / 1e12,
                              "gave_up": c["gave_up"], "stream_bytes": c["stream_bytes"]}))
        return
    if args.stream_only:
        # the product's beside shape: one 2-wave block per CU (di_pair_stream's default)
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        t, c = queue_run("stream", cus, 2)
        print(json.dumps({"what": "di_pair_stream (bounded nt stores)", "blocks": cus, "waves": 2, "jobs_per_launch": args.jobs,
                          "launches": 4, "us_per_job": 1e6 * t / args.jobs, "tb_s": job_bytes * args.jobs / t / 1e12}))
        return
    for blocks, waves in ((256, 2), (512, 1), (128, 4), (256, 4), (128, 8), (64, 4)):
        t, c = queue_run("stream", blocks, waves)
        out.append({"what": "di_pair_stream (bounded nt stores)", "blocks": blocks, "waves": waves,
                    "us_per_job": 1e6 * t / args.jobs, "tb_s": job_bytes * args.jobs / t / 1e12, "gave_up": c["gave_up"]})
    for blocks, waves in ((0, 8), (0, 4)):
        t, c = queue_run("help", blocks, waves)
        out.append({"what": "di_pair_help (plain stores)", "blocks": blocks or "CUs", "waves": waves,
                    "us_per_job": 1e6 * t / args.jobs, "tb_s": job_bytes * args.jobs / t / 1e12})
    for beside in (0, 1):
        launch = _lib.DiPairLaunch(_lib.DI_PAIR_ROWS, 0 if not beside else 128, 8 if not beside else 4, beside)

        def fn():
            for j in range(args.jobs):
                _lib.check(lib.di_pair_tensor(_lib.DI_BF16, ctypes.c_void_p(d_descs.data_ptr()), M, L, L, H, 1,
                                              ctypes.c_void_p(hT[j % 2].data_ptr()), ctypes.c_void_p(hT[j % 2].data_ptr()),
                                              n_rows, ctypes.byref(launch), ctypes.c_void_p(sinks[j % 2].data_ptr()), st),
                           "pair")
        t = timed(fn)
        out.append({"what": f"di_pair_tensor rows beside={beside}", "blocks": launch.blocks or "CUs",
                    "waves": launch.waves_per_block, "us_per_job": 1e6 * t / args.jobs,
                    "tb_s": job_bytes * args.jobs / t / 1e12})
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
