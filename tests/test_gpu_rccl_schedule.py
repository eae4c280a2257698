"""The overlapped schedule inside an RCCL process (round-5 verdict, Weak #1).

Every N > 1 rank of bench.py runs in a process with an ``nccl`` process group (torchrun). In round 5
that process configuration collapsed the schedule: the persistent pair-stream launch shared a
hardware queue with the GeoT stream, sat in front of the launches that signal it, and every stream
wave waited out its patience (bench.py --dist: 3767 complexes/s, gave_up 1024, stream_bytes 0).

Here a fresh process creates a world-size-1 ``nccl`` group first (as bench.py's dist_setup does,
communicator and its streams before any schedule stream), then runs three steps of C3 micro-batches
(8 complexes of 2 x 1000 residues each, 8 micro-batches per step: 24 jobs) through
``OverlappedSchedule`` with its default streams (pipeline.schedule_streams: hardware queues of
their own). Asserted: the streams run concurrently (di_streams_concurrent), no stream wave gave up,
the help launches wrote <= 5 % of the bytes, and every pair tensor of every job is bit-exact (the
outer concat of the GPU's own node features, deepinteract_utils.py:158-172). Whether the round-5
streams (torch's NULL stream + a pool stream) run concurrently in the same process is printed as a
diagnostic, not asserted.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

M, N_RES, K, DISTINCT, PER_STEP, STEPS = 8, 1000, 20, 3, 8, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        dist.barrier()  # the communicator exists before any stream of the schedule, as in bench.py
        from deepinteract_amd import synth
        from deepinteract_amd.builder import build_graph_batch
        from deepinteract_amd.engine import GeoTEngine
        from deepinteract_amd.graph import select_graphs
        from deepinteract_amd.pipeline import OverlappedSchedule, streams_concurrent
        from deepinteract_amd.weights import seeded_state_dict

        out = {"backend": dist.get_backend()}
        # round 5's streams in this process: the NULL stream and a torch pool stream
        out["null_and_pool_stream_concurrent"] = streams_concurrent(torch.cuda.Stream(), torch.cuda.current_stream())

        eng = GeoTEngine(seeded_state_dict(0, with_head=False), "bf16")
        eng.fuse_embed_init, eng.split_node = True, False  # bench.py's overlapped defaults
        n_cx = M * DISTINCT
        chains = [c for j in range(n_cx) for c in synth.synthetic_complex(1700 + j, N_RES, N_RES)]
        pool = build_graph_batch(chains, k=K, nbr_seeds=list(range(1, 2 * n_cx + 1)))
        distinct = [select_graphs(pool, range(2 * M * m, 2 * M * (m + 1))) for m in range(DISTINCT)]
        gb0 = distinct[0]
        h1r = [gb0.node_off[2 * j] for j in range(M)]
        h2r = [gb0.node_off[2 * j + 1] for j in range(M)]
        ref_h = []
        for gb in distinct:
            h, _ = eng.forward(gb)
            ref_h.append(h)
        torch.cuda.synchronize()
        mbs = [distinct[m % DISTINCT] for m in range(PER_STEP)]
        n_jobs = STEPS * PER_STEP
        numel = M * 2 * 128 * N_RES * N_RES
        sinks = [torch.empty(numel, dtype=torch.bfloat16, device="cuda") for _ in range(n_jobs)]
        sch = OverlappedSchedule(eng, mbs, h1r, h2r, [N_RES] * M, [N_RES] * M, sinks, ring=16, help_every=4,
                                 patience_ms=20.0)
        out["mode"], out["concurrent"] = sch.mode, sch.concurrent
        for _ in range(STEPS):
            sch.step()
        sch.finish()
        torch.cuda.synchronize()
        cnt = sch.check(allow_gave_up=True)
        out["counters"] = cnt
        bad = []
        for j in range(n_jobs):
            h = ref_h[(j % PER_STEP) % DISTINCT]
            for cx, t in enumerate(sch.views(j)):
                a, b = h[h1r[cx]:h1r[cx] + N_RES], h[h2r[cx]:h2r[cx] + N_RES]
                if not (torch.equal(t[0, :128], a.t().unsqueeze(2).expand(128, N_RES, N_RES))
                        and torch.equal(t[0, 128:], b.t().unsqueeze(1).expand(128, N_RES, N_RES))):
                    bad.append((j, cx))
        out["bad"], out["n_jobs"] = bad, n_jobs
        out["expected_bytes"] = n_jobs * M * 256 * N_RES * N_RES * 2
        del sinks, sch
        dist.destroy_process_group()
        q.put((out, None))
    except Exception as exc:  # reported to the parent instead of hanging it
        q.put((None, repr(exc)))


def test_overlapped_schedule_in_rccl_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        out, err = q.get(timeout=300)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert err is None, err
    cnt = out["counters"]
    tot = cnt["stream_bytes"] + cnt["help_bytes"]
    print("RCCL process: backend", out["backend"], "| NULL + pool stream concurrent:",
          out["null_and_pool_stream_concurrent"], "| schedule mode", out["mode"], "| counters", cnt,
          f"| help share {cnt['help_bytes'] / max(tot, 1):.4f}")
    assert out["backend"] == "nccl"
    assert out["concurrent"] and out["mode"] == "overlapped"
    assert cnt["error"] == 0 and cnt["gave_up"] == 0, cnt
    assert cnt["signalled"] == out["n_jobs"], cnt
    assert tot == out["expected_bytes"], cnt
    assert cnt["help_bytes"] <= 0.05 * tot, cnt
    assert out["bad"] == [], out["bad"]
    assert p.exitcode == 0
