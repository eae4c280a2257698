"""Complex-sharded data parallelism over torch.distributed (RCCL on ROCm, gloo in CPU tests).

SURVEY.md §8e: complexes are independent (eval-mode BatchNorm, replicated weights), so the
forward shards by complex with no exchange; the only collective is ONE all-gather of the
contact maps after the head (the reference has no multi-GPU inference; its predict path is
single-node DP, lit_model_predict_docker.py:183, producing per-complex maps as
lit_model_predict.py:236-239 does).

* ``shard`` — contiguous shards: rank r owns complexes [b_r, b_{r+1}), the boundaries chosen so
  every rank's summed cost (L1*L2 pair work + (L1+L2)*k edge work) is as even as a contiguous
  split allows; every rank computes the same plan from the sizes alone.
* ``local_order`` — a rank's complexes in size-sorted order, so micro-batches group similar
  sizes (varlen work balanced inside each launch).
* ``all_gather_maps`` — packs each rank's [L1,L2] maps into one flat buffer (padded to the
  largest rank's element count) and issues a single ``all_gather_into_tensor``; on xGMI one big
  collective beats many small ones (7 point-to-point links per GPU). dtype and device are
  arguments every rank passes identically, so a rank that owns no complex still sends a
  buffer of the agreed type.
* ``predict_sharded`` — the C4 driver: shard -> micro-batched forward (graph build, GeoT,
  pair tensor / head prologue, head, contact probabilities) -> the maps on every rank, gathered
  either chunked (default, SURVEY.md §8e: round c gathers every rank's c-th micro-batch of maps
  with an asynchronous ``all_gather_into_tensor`` issued as soon as they exist, so the collective
  of round c runs on the process group's stream while round c+1 computes) or ONCE after the last
  micro-batch (``all_gather_maps``). Both return bit-identical maps.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch
import torch.distributed as dist


def complex_cost(l1: int, l2: int, k: int = 20) -> int:
    return l1 * l2 + k * (l1 + l2)


def shard(sizes: Sequence[tuple], world: int, k: int = 20):
    """sizes: (L1, L2) per complex -> per rank, the contiguous list of its complex indices.

    Boundary b_r is the first index whose cost prefix reaches r/world of the total, so each
    shard's cost is within one complex of the even share."""
    n = len(sizes)
    cost = [complex_cost(a, b, k) for a, b in sizes]
    total = float(sum(cost))
    bounds, acc, i = [0], 0.0, 0
    for r in range(1, world):
        target = total * r / world
        while i < n and acc + cost[i] / 2.0 <= target:
            acc += cost[i]
            i += 1
        bounds.append(i)
    bounds.append(n)
    return [list(range(bounds[r], bounds[r + 1])) for r in range(world)]


def local_order(sizes: Sequence[tuple], indices: Sequence[int]):
    """A rank's complexes, largest first (stable), for size-grouped micro-batches."""
    return sorted(indices, key=lambda i: (-(sizes[i][0] * sizes[i][1]), i))


def all_gather_maps(local_maps: Sequence[torch.Tensor], plan, sizes, dtype: torch.dtype,
                    device, group=None):
    """Gather every rank's contact maps; returns the maps of ALL complexes in global order.

    local_maps: this rank's maps in the order of plan[rank]; dtype / device: the wire format,
    identical on every rank (RCCL needs matching dtypes and sizes on all ranks)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(plan) != world:
        raise ValueError(f"plan has {len(plan)} shards for a world of {world}")
    counts = [sum(sizes[i][0] * sizes[i][1] for i in p) for p in plan]
    width = max(max(counts), 1)
    send = torch.zeros(width, dtype=dtype, device=device)
    if len(local_maps) != len(plan[rank]):
        raise ValueError(f"rank {rank}: {len(local_maps)} maps for {len(plan[rank])} planned complexes")
    if len(local_maps):
        flat = torch.cat([m.reshape(-1).to(device=device, dtype=dtype) for m in local_maps])
        if flat.numel() != counts[rank]:
            raise ValueError(f"rank {rank}: maps hold {flat.numel()} elements, plan says {counts[rank]}")
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


def gpu_forward(model, k: int = 20, seed: int = 0):
    """The per-micro-batch forward of ``predict_sharded`` on the HIP path: on-device graph build
    (deepinteract_amd.builder) -> LitGINI.predict_batch -> contact probabilities. Complex i's
    chains draw their neighbour-edge ids as torch.manual_seed(seed + 2i + s) would (s = 0, 1), so
    the maps do not depend on how the complexes are sharded or micro-batched. out (optional): one
    [L1, L2] tensor per complex -- the chunked gather's send slices -- that receive the maps (the
    softmax output written straight into the collective's buffer, in its wire dtype)."""
    from .builder import build_graph_batch

    def fn(complexes, ids, out=None):
        chains = [c for pair in complexes for c in pair]
        dev = model.engine.device
        gb = build_graph_batch(chains, k=k, device=dev, node_count_limit=model.cfg.node_count_limit,
                               nbr_seeds=[seed + 2 * i + s for i in ids for s in (0, 1)])
        with torch.no_grad():
            _, probs = model.predict_batch(gb, [(2 * j, 2 * j + 1) for j in range(len(complexes))])
            if out is not None:
                for dst, p in zip(out, probs):
                    dst.copy_(p)
                return out
        return probs

    return fn


def gather_rounds(sizes: Sequence[tuple], plan, micro_batch: int):
    """The chunked all-gather's schedule, computed by every rank from the sizes alone: round c holds
    micro-batch c of every rank (its size-sorted local order cut into micro_batch-sized pieces; a
    rank with fewer micro-batches contributes nothing to the later rounds). Returns per round
    (per-rank complex lists, the round's per-rank buffer width in elements)."""
    mbs = []
    for p in plan:
        order = local_order(sizes, p)
        mbs.append([order[s:s + micro_batch] for s in range(0, len(order), micro_batch)])
    rounds = []
    for c in range(max((len(m) for m in mbs), default=0)):
        members = [m[c] if c < len(m) else [] for m in mbs]
        width = max(max(sum(sizes[i][0] * sizes[i][1] for i in ids) for ids in members), 1)
        rounds.append((members, width))
    return rounds


class ChunkedGather:
    """Round-by-round asynchronous all-gather of contact maps (chunked and overlapped
    with compute). Every round's send and receive buffers are allocated up front (sizes are known
    from the plan), and ``slots(c)`` hands out this rank's [L1, L2] slices of round c's send buffer
    for the forward to write its maps into (gpu_forward's ``out``): the compute stream runs no pack,
    pad or cast kernels. ``put(c)`` issues ``all_gather_into_tensor(..., async_op=True)`` -- on
    RCCL it runs on the process group's own stream, which waits for the work already queued on the
    current stream (one event), so the next micro-batch's kernels, issued right after, overlap it;
    ``finish()`` waits for every round and returns the maps of all complexes in global order (views
    of the rounds' receive buffers)."""

    def __init__(self, sizes, plan, micro_batch, dtype, device, group=None):
        self.sizes, self.dtype, self.device, self.group = sizes, dtype, device, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.rounds = gather_rounds(sizes, plan, micro_batch)
        # padding of a round's send buffer is never read by a receiver; zeroed once for determinism
        self.send = [torch.zeros(width, dtype=dtype, device=device) for _, width in self.rounds]
        self.recv = [torch.empty(self.world * width, dtype=dtype, device=device) for _, width in self.rounds]
        self.pending = []

    def slots(self, c):
        """This rank's maps of round c as [L1, L2] views of the round's send buffer (member order)."""
        views, off = [], 0
        for i in self.rounds[c][0][self.rank]:
            l1, l2 = self.sizes[i]
            views.append(self.send[c][off:off + l1 * l2].view(l1, l2))
            off += l1 * l2
        return views

    def put(self, c, maps=None):
        """Issue round c's collective. maps (optional): this rank's maps of the round, copied into the
        send slices (for a forward that did not write them there itself)."""
        mine = self.rounds[c][0][self.rank]
        if maps is not None:
            if len(maps) != len(mine):
                raise ValueError(f"rank {self.rank}: {len(maps)} maps for round {c}'s {len(mine)} complexes")
            for dst, m in zip(self.slots(c), maps):
                if dst.data_ptr() != m.data_ptr():
                    dst.copy_(m)
        self._issue(c)

    def _issue(self, c):
        work = dist.all_gather_into_tensor(self.recv[c], self.send[c], group=self.group, async_op=True)
        self.pending.append((c, self.recv[c], self.send[c], work))

    def finish(self):
        # rounds in which this rank has no micro-batch still take part (every rank issues every round)
        done = {c for c, *_ in self.pending}
        for c in range(len(self.rounds)):
            if c not in done:
                self._issue(c)
        out = [None] * len(self.sizes)
        for c, recv, _send, work in sorted(self.pending, key=lambda t: t[0]):
            work.wait()
            members, width = self.rounds[c]
            for r, ids in enumerate(members):
                off = r * width
                for i in ids:
                    l1, l2 = self.sizes[i]
                    out[i] = recv[off:off + l1 * l2].view(l1, l2)
                    off += l1 * l2
        self.pending = []
        return out


def predict_sharded(complexes: Sequence, forward: Callable, micro_batch: int = 8, dtype=torch.float32,
                    device=None, group=None, gather: str = "chunked"):
    """C4 driver: every rank runs ``forward`` over its contiguous shard of
    ``complexes`` in size-sorted micro-batches; every complex's contact map ends on every rank.

    complexes: per complex a (chain1, chain2) pair of builder inputs (dicts with backbone
    [N,4,3], amide_norm [N,3], dips [N,106]); forward(batch, ids) -> list of [L1, L2] maps for
    the complexes ``batch`` (global indices ``ids``); a forward that takes ``out=`` (gpu_forward)
    writes them straight into the chunked gather's send slices.
    gather: "chunked" (default) -- one asynchronous all-gather per micro-batch round, overlapped
    with the next round's compute (ChunkedGather); "once" -- ONE all-gather after the last
    micro-batch (all_gather_maps); "none" -- no collective, this rank's maps only (timing the
    compute alone). Returns the maps (global order; None for other ranks' complexes with "none")
    and the plan."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [(int(len(c[0]["backbone"])), int(len(c[1]["backbone"]))) for c in complexes]
    plan = shard(sizes, world)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
            else torch.device("cpu")
    if gather not in ("chunked", "once", "none"):
        raise ValueError(f"gather {gather!r}: one of chunked, once, none")
    chunks = ChunkedGather(sizes, plan, micro_batch, dtype, device, group) if gather == "chunked" else None
    mine = local_order(sizes, plan[rank])
    maps = {}
    import inspect
    takes_out = "out" in inspect.signature(forward).parameters
    for c, s in enumerate(range(0, len(mine), micro_batch)):
        ids = mine[s:s + micro_batch]
        if chunks is not None and takes_out:
            got = list(forward([complexes[i] for i in ids], ids, out=chunks.slots(c)))
        else:
            got = list(forward([complexes[i] for i in ids], ids))
        for i, m in zip(ids, got):
            if tuple(m.shape) != sizes[i]:
                raise ValueError(f"complex {i}: map {tuple(m.shape)} != {sizes[i]}")
            maps[i] = m
        if chunks is not None:
            chunks.put(c, got)
    if gather == "chunked":
        return chunks.finish(), plan
    if gather == "none":
        return [maps.get(i) for i in range(len(sizes))], plan
    return all_gather_maps([maps[i] for i in plan[rank]], plan, sizes, dtype, device, group), plan
