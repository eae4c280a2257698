"""Debug: the bf16 di_node_layer vs the split form (di_node_aggregate + di_node_update) on random CSRs;
prints where they differ (node rows mod the 32-destination tile, feature blocks).
usage (GPU box): python tools/debug/node_sp_dbg.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepinteract_amd import _lib  # noqa: E402
from deepinteract_amd.engine import GeoTEngine  # noqa: E402
from deepinteract_amd.weights import seeded_state_dict  # noqa: E402


def run(n, deg_lo, deg_hi, final, seed=0):
    lib = _lib.load()
    eng = GeoTEngine(seeded_state_dict(0), "bf16")
    nm, nv = eng.packed.node[1 if final else 0]
    g = torch.Generator().manual_seed(seed)
    deg = torch.randint(deg_lo, deg_hi + 1, (n,), generator=g)
    in_ptr = torch.zeros(n + 1, dtype=torch.int32)
    in_ptr[1:] = torch.cumsum(deg, 0)
    E = int(in_ptr[-1])
    src = torch.randint(0, n, (E,), generator=g, dtype=torch.int32)
    alpha = torch.exp(torch.empty(E, 4).uniform_(-5, 5, generator=g))
    dev = torch.device("cuda")
    qkv = torch.randn(n, 384, generator=g).to(torch.bfloat16).to(dev)
    h_in = torch.randn(n, 128, generator=g).to(torch.bfloat16).to(dev)
    d_src, d_ptr, d_alpha = src.to(dev), in_ptr.to(dev), alpha.to(dev)
    cg = _lib.DiGraph(n, E, d_src.data_ptr(), None, None, None, d_ptr.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    outs = []
    for split in (False, True):
        h_out = torch.full((n, 128), float("nan"), dtype=torch.bfloat16, device=dev)
        q_out = None if final else torch.full((n, 384), float("nan"), dtype=torch.bfloat16, device=dev)
        hT = torch.full((128, n), float("nan"), dtype=torch.bfloat16, device=dev) if final else None
        if split:
            attn = torch.empty(n, 128, device=dev)
            assert lib.di_node_aggregate(ctypes.byref(cg), _lib.DI_BF16, p(d_alpha), p(qkv), p(attn), st) == 0
            assert lib.di_node_update(ctypes.byref(cg), _lib.DI_BF16, int(final), p(attn), p(h_in), p(nm), p(nv),
                                      p(h_out), p(q_out), p(hT), st) == 0
        else:
            assert lib.di_node_layer(ctypes.byref(cg), _lib.DI_BF16, int(final), p(d_alpha), p(h_in), p(qkv), p(nm),
                                     p(nv), p(h_out), p(q_out), p(hT), st) == 0
        torch.cuda.synchronize()
        outs.append((h_out.float().cpu(), None if q_out is None else q_out.float().cpu()))
    (h0, q0), (h1, q1) = outs
    bad = (h0 != h1) & ~(torch.isnan(h0) & torch.isnan(h1))
    rows = bad.any(1).nonzero().flatten()
    print(f"n={n} deg {deg_lo}-{deg_hi} final={final}: h rows differing {len(rows)} / {n}; nan in sp {torch.isnan(h0).sum().item()}")
    if len(rows):
        r = rows[:64]
        print("  rows", r.tolist()[:32])
        print("  rows mod 32", sorted(set((r % 32).tolist())))
        cols = bad[rows].any(0).nonzero().flatten()
        print("  feature blocks", sorted(set((cols // 16).tolist())))
        print("  max abs diff", (h0 - h1)[bad].abs().max().item())
    if q0 is not None:
        qb = (q0 != q1)
        print(f"  qkv rows differing {qb.any(1).sum().item()}")


if __name__ == "__main__":
    for n in (96, 512, 1000):
        for final in (False, True):
            run(n, 20, 20, final)
    run(512, 0, 40, False)
    run(9613, 0, 40, True)
