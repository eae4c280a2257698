"""Complex-sharded data parallelism over torch.distributed (RCCL on ROCm, gloo in CPU tests).

SURVEY.md §8e: complexes are independent (eval-mode BatchNorm, replicated weights), so the
forward shards by complex with no exchange; the only collective is ONE all-gather of the
contact maps after the head (the reference has no multi-GPU inference; its predict path is
single-node DP, lit_model_predict_docker.py:183).

* ``shard`` — size-balanced contiguous-by-rank assignment (longest-processing-time greedy on
  L1*L2 + edges, so varlen complexes spread evenly); every rank computes the same plan.
* ``all_gather_maps`` — packs each rank's [L1,L2] maps into one flat buffer (padded to the
  largest rank's element count) and issues a single ``all_gather_into_tensor``; on xGMI one big
  collective beats many small ones (7 point-to-point links per GPU).
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.distributed as dist


def shard(sizes: Sequence[tuple], world: int):
    """sizes: (L1, L2) per complex -> list (per rank) of complex indices, cost-balanced."""
    cost = [l1 * l2 + 20 * (l1 + l2) for l1, l2 in sizes]
    order = sorted(range(len(sizes)), key=lambda i: (-cost[i], i))
    load = [0] * world
    plan = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda q: (load[q], q))
        plan[r].append(i)
        load[r] += cost[i]
    return [sorted(p) for p in plan]


def all_gather_maps(local_maps: Sequence[torch.Tensor], plan, sizes, group=None):
    """Gather every rank's contact maps; returns the maps of ALL complexes in global order."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [sum(sizes[i][0] * sizes[i][1] for i in p) for p in plan]
    width = max(max(counts), 1)
    ref = local_maps[0] if len(local_maps) else None
    dtype = ref.dtype if ref is not None else torch.float32
    device = ref.device if ref is not None else (torch.device("cuda") if dist.get_backend(group) == "nccl"
                                                  else torch.device("cpu"))
    send = torch.zeros(width, dtype=dtype, device=device)
    if len(local_maps):
        flat = torch.cat([m.reshape(-1) for m in local_maps])
        assert flat.numel() == counts[rank], (flat.numel(), counts[rank])
        send[:flat.numel()] = flat
    recv = torch.empty(world * width, dtype=dtype, device=device)
    dist.all_gather_into_tensor(recv, send, group=group)
    out = [None] * len(sizes)
    for r, p in enumerate(plan):
        off = r * width
        for i in p:
            l1, l2 = sizes[i]
            out[i] = recv[off:off + l1 * l2].view(l1, l2)
            off += l1 * l2
    return out
