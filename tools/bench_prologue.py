"""Head-prologue benchmark: ELU(inorm_1(conv2d_1(T))) for a micro-batch of C3
complexes (2 x 1000 residues, bf16), fused on HIP (di_head_prologue: T never materialised) vs the
unfused path (HIP pair tensor T, then MIOpen conv2d_1 + InstanceNorm + ELU in torch). Prints one
JSON line; the fused kernel's roofline is its written bytes (C * L1 * L2 * 2 per complex) over
its HIP-event time.

usage: python tools/bench_prologue.py [--complexes 8] [--reps 10]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from deepinteract_amd.engine import HeadPrologueOp, PairTensorOp  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--complexes", type=int, default=8)
    ap.add_argument("--residues", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    M, L, H, C = a.complexes, a.residues, 128, 128
    dev = torch.device("cuda")
    torch.manual_seed(0)
    h = torch.randn(2 * M * L, H, device=dev).to(torch.bfloat16)
    w = torch.randn(C, 2 * H, 1, 1, device=dev) / 16
    b, g, bt = torch.randn(C, device=dev) * 0.1, 1 + 0.1 * torch.randn(C, device=dev), 0.1 * torch.randn(C, device=dev)
    h1r = [2 * L * m for m in range(M)]
    h2r = [2 * L * m + L for m in range(M)]
    ls = [L] * M
    pro = HeadPrologueOp(w, b, g, bt, 1e-6, dev)
    out = torch.empty(M * C * L * L, dtype=torch.bfloat16, device=dev)
    t_fused = timed(lambda: pro(h, h1r, h2r, ls, ls, out=out), a.reps)

    pair = PairTensorOp(dev, kernel="rows")
    hT = h.t().contiguous()
    tbuf = torch.empty(M * 2 * H * L * L, dtype=torch.bfloat16, device=dev)
    wb = w.to(torch.bfloat16)

    def unfused():
        _, views = pair(h, h1r, h2r, ls, ls, out=tbuf, hT=hT)
        t = tbuf.view(M, 2 * H, L, L)
        x = F.conv2d(t, wb, b.to(torch.bfloat16))
        x = F.instance_norm(x, weight=g.to(torch.bfloat16), bias=bt.to(torch.bfloat16), eps=1e-6)
        return F.elu(x)
    t_unfused = timed(unfused, max(2, a.reps // 3))

    # agreement of the two paths on this batch (bf16 both): max-abs err / max-abs
    ref = unfused().float()
    got = out.view(M, C, L, L).float()
    err = float((got - ref).abs().max() / ref.abs().max())
    byts = M * C * L * L * 2
    gbs = byts / (t_fused * 1e-6) / 1e9
    print(json.dumps({
        "op": "head prologue ELU(inorm_1(conv2d_1(T)))", "complexes": M, "residues": [L, L], "dtype": "bf16",
        "fused_us_per_batch": round(t_fused, 1), "unfused_us_per_batch": round(t_unfused, 1),
        "speedup": round(t_unfused / t_fused, 2),
        "fused_roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                           "frac": round(gbs / 8000.0, 4), "algorithmic_bytes_per_complex": C * L * L * 2},
        "unfused_path": "HIP pair tensor (rows) + torch/MIOpen conv2d_1 + instance_norm + elu (bf16)",
        "rel_err_vs_unfused_bf16": err,
    }), flush=True)


if __name__ == "__main__":
    main()
