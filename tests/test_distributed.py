"""World-size-2 gloo tests of the complex-sharded path (CPU): sharding plan and the single
all-gather of contact maps."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deepinteract_amd.distributed import all_gather_maps, shard


def test_shard_balanced_and_complete():
    sizes = [(1000, 1000)] * 7 + [(145, 145), (256, 256), (2000, 300)]
    for world in (1, 2, 4, 8):
        plan = shard(sizes, world)
        flat = sorted(i for p in plan for i in p)
        assert flat == list(range(len(sizes)))
        if world <= 7:
            assert all(len(p) >= 1 for p in plan)
    plan = shard([(100, 100)] * 16, 4)
    assert [len(p) for p in plan] == [4, 4, 4, 4]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sizes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = shard(sizes, world)
        maps = [torch.full((l1, l2), float(i)) + torch.arange(l2).float() / 1000
                for i, (l1, l2) in enumerate(sizes) if i in plan[rank]]
        maps = [maps[j] for j in range(len(maps))]
        got = all_gather_maps(maps, plan, sizes)
        ok = all(torch.equal(got[i], torch.full(sizes[i], float(i)) + torch.arange(sizes[i][1]).float() / 1000)
                 for i in range(len(sizes)))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_all_gather_contact_maps_gloo(world):
    sizes = [(7, 5), (3, 9), (12, 12), (1, 4), (6, 6)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res
