"""C4 (BASELINE configs[3]) on the GPU: the complex-sharded driver with the REAL HIP forward.

Two gloo ranks share cuda:0. Each runs ``distributed.predict_sharded(cx, gpu_forward(model),
micro_batch=2)`` over seven synthetic complexes of mixed sizes, one of them C4's own 2x1000: the
device builder with torch-seeded neighbour ids, fp32 GeoT, the pair tensor, the fp32 head with GEMM
convolutions (``precise_head``) and contact probabilities; then the maps gathered (chunked: one
asynchronous all-gather per micro-batch round). Every rank must end with every complex's map,
bit-identical to a single-process ``model.predict_batch`` over the same device-built graphs (same
seeds -> same ids, and every kernel computes a chain independently of its batch-mates).

RCCL itself: one process with a world-size-1 ``nccl`` process group on cuda:0 (the backend
bench.py initialises under torchrun) runs ``predict_sharded(..., device="cuda")`` in both gather
modes and ``all_gather_maps`` with fp32 and bf16 maps on the device.

The reference's multi-device predict is data parallel (lit_model_predict_docker.py:183) and each
map is softmax(logits)[:, 1] (lit_model_predict.py:236-239).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = [(145, 145), (256, 256), (300, 500), (145, 256), (200, 180), (256, 145), (1000, 1000)]
SEED = 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    from deepinteract_amd.modules import LitGINI
    from deepinteract_amd.weights import seeded_state_dict
    model = LitGINI(dtype="f32", precise_head=True).to("cuda:0").eval()
    return model.load_reference_state_dict(seeded_state_dict(0))


def _complexes():
    from deepinteract_amd import synth
    return [synth.synthetic_complex(900 + i, a, b) for i, (a, b) in enumerate(SIZES)]


def _single_process_maps(model, cx):
    """predict_batch over all complexes in one device batch, ids seeded as gpu_forward seeds them."""
    from deepinteract_amd.builder import build_graph_batch
    chains = [c for pair in cx for c in pair]
    gb = build_graph_batch(chains, k=20, device="cuda:0", node_count_limit=model.cfg.node_count_limit,
                           nbr_seeds=[SEED + 2 * i + s for i in range(len(cx)) for s in (0, 1)])
    with torch.no_grad():
        _, probs = model.predict_batch(gb, [(2 * j, 2 * j + 1) for j in range(len(cx))])
    return [p.float().cpu() for p in probs]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from deepinteract_amd.distributed import gpu_forward, predict_sharded
        model = _model()
        cx = _complexes()
        maps, plan = predict_sharded(cx, gpu_forward(model, k=20, seed=SEED), micro_batch=2,
                                     dtype=torch.float32, device="cpu")
        torch.cuda.synchronize()
        ref = _single_process_maps(model, cx)
        diffs = [float((m.float() - r).abs().max()) for m, r in zip(maps, ref)]
        equal = [bool(torch.equal(m.float(), r)) for m, r in zip(maps, ref)]
        shapes = [tuple(m.shape) for m in maps]
        in_range = all(0.0 <= float(m.min()) and float(m.max()) <= 1.0 for m in maps)
        q.put((rank, equal, diffs, shapes, [len(p) for p in plan], in_range, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as exc:  # reported to the parent instead of hanging it
        q.put((rank, None, None, None, None, None, repr(exc)))


def test_c4_predict_sharded_two_ranks_on_gpu_bit_identical():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=400) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, equal, diffs, shapes, plan, in_range, err in res:
        assert err is None, f"rank {rank}: {err}"
        print(f"rank {rank}: plan sizes {plan}, max |sharded - single-process| per complex {diffs}")
        assert shapes == SIZES, shapes
        assert sum(plan) == len(SIZES) and min(plan) >= 1
        assert in_range
        assert all(equal), (rank, diffs)
    assert [p.exitcode for p in procs] == [0, 0]


def _worker_nccl1(port, q):
    """World-size-1 RCCL group on cuda:0: the device-side gather paths of predict_sharded."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        from deepinteract_amd.distributed import all_gather_maps, gpu_forward, predict_sharded, shard
        model = _model()
        cx = _complexes()[:6]
        sizes = SIZES[:6]
        ref = _single_process_maps(model, cx)
        out = {"backend": dist.get_backend()}
        for gather in ("chunked", "once"):
            maps, plan = predict_sharded(cx, gpu_forward(model, k=20, seed=SEED), micro_batch=2,
                                         dtype=torch.float32, device="cuda", gather=gather)
            torch.cuda.synchronize()
            out[gather] = (all(m.is_cuda for m in maps),
                           [bool(torch.equal(m.float().cpu(), r)) for m, r in zip(maps, ref)])
        plan = shard(sizes, 1)
        for dt in (torch.float32, torch.bfloat16):
            got = all_gather_maps([r.cuda() for r in ref], plan, sizes, dt, "cuda")
            torch.cuda.synchronize()
            out[str(dt)] = [bool(g.dtype == dt and g.is_cuda and torch.equal(g.cpu(), r.to(dt))) for g, r in zip(got, ref)]
        dist.destroy_process_group()
        q.put((out, None))
    except Exception as exc:
        q.put((None, repr(exc)))


def test_rccl_world1_predict_sharded_and_gather_on_device():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_nccl1, args=(_free_port(), q))
    p.start()
    try:
        out, err = q.get(timeout=300)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert err is None, err
    print("world-size-1 RCCL:", out)
    assert out["backend"] == "nccl"
    for gather in ("chunked", "once"):
        on_dev, equal = out[gather]
        assert on_dev and all(equal), (gather, equal)
    assert all(out["torch.float32"]) and all(out["torch.bfloat16"])
    assert p.exitcode == 0
