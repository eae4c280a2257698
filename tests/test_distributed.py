"""World-size-2/3 gloo tests of the complex-sharded path (CPU): the contiguous sharding plan, the
single all-gather of contact maps (incl. a rank that owns no complex, bf16 maps), the chunked
round-by-round asynchronous all-gather, and the composed C4 driver ``predict_sharded`` with a CPU
stand-in for the GPU forward (both gather modes: bit-identical maps)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deepinteract_amd.distributed import (all_gather_maps, complex_cost, gather_rounds, local_order, predict_sharded,
                                          shard)


def test_shard_contiguous_balanced_and_complete():
    sizes = [(1000, 1000)] * 7 + [(145, 145), (256, 256), (2000, 300)]
    for world in (1, 2, 4, 8, 16):
        plan = shard(sizes, world)
        assert len(plan) == world
        flat = [i for p in plan for i in p]
        assert flat == list(range(len(sizes)))          # contiguous, in order, complete
        if world <= 7:
            assert all(len(p) >= 1 for p in plan)
    plan = shard([(100, 100)] * 16, 4)
    assert [len(p) for p in plan] == [4, 4, 4, 4]
    # cost balance: every shard within one (largest) complex of the even share
    rng = np.random.default_rng(0)
    sizes = [(int(a), int(b)) for a, b in rng.integers(50, 1500, size=(200, 2))]
    cost = [complex_cost(a, b) for a, b in sizes]
    for world in (2, 3, 8):
        plan = shard(sizes, world)
        loads = [sum(cost[i] for i in p) for p in plan]
        assert max(loads) - sum(cost) / world <= max(cost)


def test_local_order_size_sorted():
    sizes = [(10, 10), (30, 30), (20, 20), (30, 30)]
    assert local_order(sizes, [0, 1, 2, 3]) == [1, 3, 2, 0]


def test_gather_rounds_cover_every_complex_once():
    """Round c holds micro-batch c of every rank; uneven ranks contribute nothing to later rounds;
    each round's width is its largest rank's element count."""
    sizes = [(30, 22), (25, 25), (40, 21), (21, 33), (28, 30), (10, 10), (12, 9)]
    for world in (1, 2, 3, 8):
        plan = shard(sizes, world)
        rounds = gather_rounds(sizes, plan, 2)
        seen = [i for members, _ in rounds for ids in members for i in ids]
        assert sorted(seen) == list(range(len(sizes)))
        for members, width in rounds:
            assert len(members) == world
            assert width == max(max(sum(sizes[i][0] * sizes[i][1] for i in ids) for ids in members), 1)
        for r in range(world):
            mine = [i for members, _ in rounds for i in members[r]]
            assert mine == local_order(sizes, plan[r])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _map_of(i, l1, l2, dtype=torch.float32):
    return (torch.full((l1, l2), float(i)) + torch.arange(l2).float() / 1000).to(dtype)


def _worker_gather(rank, world, port, sizes, dtype, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = shard(sizes, world)
        maps = [_map_of(i, *sizes[i], dtype) for i in plan[rank]]
        got = all_gather_maps(maps, plan, sizes, dtype=dtype, device="cpu")
        ok = all(got[i].dtype == dtype and torch.equal(got[i], _map_of(i, *sizes[i], dtype))
                 for i in range(len(sizes)))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("sizes,dtype", [
    ([(7, 5), (3, 9), (12, 12), (1, 4), (6, 6)], torch.float32),
    ([(9, 4)], torch.bfloat16),            # world > complexes: rank 1 owns nothing, still sends bf16
])
def test_all_gather_contact_maps_gloo(sizes, dtype):
    res = _spawn(_worker_gather, 2, sizes, dtype)
    assert all(ok for _, ok in res), res


def _chain(n, seed):
    rng = np.random.default_rng(seed)
    return {"backbone": rng.normal(size=(n, 4, 3)).astype(np.float32),
            "amide_norm": rng.normal(size=(n, 3)).astype(np.float32),
            "dips": rng.random((n, 106)).astype(np.float32)}


def _complexes():
    lens = [(30, 22), (25, 25), (40, 21), (21, 33), (28, 30)]
    return [(_chain(a, 2 * i), _chain(b, 2 * i + 1)) for i, (a, b) in enumerate(lens)]


def _cpu_forward(batch, ids):
    """Stand-in for the GPU forward: a deterministic per-complex map from the chains' coordinates
    (independent of which rank or micro-batch computes it)."""
    out = []
    for c1, c2 in batch:
        a = torch.as_tensor(c1["backbone"][:, 1, :])
        b = torch.as_tensor(c2["backbone"][:, 1, :])
        out.append(torch.sigmoid(-torch.cdist(a, b)))
    return out


def _cpu_forward_out(batch, ids, out=None):
    """_cpu_forward writing into the caller's buffers when given (gpu_forward's contract: the chunked
    gather's send slices)."""
    maps = _cpu_forward(batch, ids)
    if out is None:
        return maps
    for dst, m in zip(out, maps):
        dst.copy_(m)
    return out


def _worker_predict(rank, world, port, gather, dtype, fwd, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cx = _complexes()
        forward = _cpu_forward_out if fwd == "out" else _cpu_forward
        maps, plan = predict_sharded(cx, forward, micro_batch=2, gather=gather, dtype=dtype)
        ref = [m.to(dtype) for m in _cpu_forward(cx, list(range(len(cx))))]
        ok = len(maps) == len(cx) and all(m.dtype == dtype and torch.equal(m, r) for m, r in zip(maps, ref))
        q.put((rank, ok, [len(p) for p in plan]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,gather,dtype", [(2, "once", torch.float32), (2, "chunked", torch.float32),
                                                (3, "chunked", torch.float32), (2, "chunked", torch.bfloat16)])
def test_predict_sharded_gloo(world, gather, dtype):
    """The composed C4 driver: contiguous shard -> size-sorted micro-batches -> forward -> the maps
    gathered once at the end or round by round with asynchronous all-gathers (world 3: ranks with
    different micro-batch counts); every rank ends with every complex's map, equal to a
    single-process run."""
    res = _spawn(_worker_predict, world, gather, dtype, "plain")
    assert all(ok for _, ok, _ in res), res
    assert sum(res[0][2]) == len(_complexes())


@pytest.mark.parametrize("world,dtype", [(2, torch.float32), (3, torch.bfloat16)])
def test_predict_sharded_chunked_forward_writes_send_slices(world, dtype):
    """The chunked gather with a forward that takes ``out=``: the maps are written straight into the
    rounds' preallocated send buffers (no pack / pad / cast on the compute stream) and gathered
    bit-identical to a single-process run."""
    res = _spawn(_worker_predict, world, "chunked", dtype, "out")
    assert all(ok for _, ok, _ in res), res
