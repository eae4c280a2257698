"""Contact-head benchmark (outside the metric): the dilated-ResNet head
(deepinteract_modules.py:1155-1248, 14 chunks x {1,2,4,8} + phase 2) on PyTorch-ROCm / MIOpen for one
C3 complex (input [1,256,L,L]), in five forms: fp32 / bf16 NCHW with torch's InstanceNorm / ELU / SE passes,
the same with those passes on HIP (head.HeadNormOps, csrc/head_ops.hip), and bf16 channels-last (NHWC). Prints one JSON line: ms per complex, TFLOP/s against the head's
algorithmic FLOPs (~3.49 M MAC per pixel) and the bf16 logits' max error relative
to the fp32 logits of the same input.

usage: python tools/bench_head.py [--residues 1000] [--reps 3]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from deepinteract_amd.head import HeadNormOps, ResNet2DInputWithOptAttention  # noqa: E402
from deepinteract_amd.weights import seeded_state_dict  # noqa: E402


def head_macs_per_px(C=128, chunks=14):
    blk = C * (C // 2) + (C // 2) * (C // 2) * 9 + (C // 2) * C  # conv 1x1, 3x3 dilated, 1x1
    n_blocks = 4 * chunks + 4 + 2  # base resnet + phase-2 resnet (1 chunk + 2 extra)
    return 2 * C * C + n_blocks * blk + 2 * C * C + C * 2  # conv2d_1 (256->128), init projs, phase2_conv


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--residues", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="comma-separated variant names (default: all)")
    a = ap.parse_args()
    L = a.residues
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    sd = seeded_state_dict(0)
    head_sd = {k[len("interact_module."):]: v for k, v in sd.items() if k.startswith("interact_module.")}
    g = torch.Generator(device="cpu").manual_seed(0)
    t = torch.randn(1, 256, L, L, generator=g).to(dev)
    flops = 2.0 * head_macs_per_px() * L * L
    out = {"workload": f"contact head, one [1,256,{L},{L}] complex", "mac_per_px": head_macs_per_px()}
    ref = None
    variants = (("f32_nchw", torch.float32, False, False), ("f32_nchw_hipnorm", torch.float32, False, True),
                ("bf16_nchw", torch.bfloat16, False, False), ("bf16_nchw_hipnorm", torch.bfloat16, False, True),
                ("bf16_nhwc", torch.bfloat16, True, False))
    for name, dt, cl, hip in variants:
        if a.only and name not in a.only.split(","):
            continue
        m = ResNet2DInputWithOptAttention().to(dev).eval()
        m.load_state_dict(head_sd)
        m.to(dtype=dt)
        if hip:
            m.use_hip_norm_ops(HeadNormOps(dev))
        x = t.to(dt)
        if cl:
            m.to(memory_format=torch.channels_last)
            x = x.contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            y = m(x).float()
            ms = timed(lambda: m(x), a.reps)
        rec = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 2)}
        if name == "f32_nchw":
            ref = y
        elif ref is None:
            pass
        else:
            rec["logits_rel_err_vs_f32"] = float((y - ref).abs().max() / ref.abs().max())
            p, pr = torch.softmax(y[0], 0)[1], torch.softmax(ref[0], 0)[1]
            rec["prob_max_abs_err_vs_f32"] = float((p - pr).abs().max())
        out[name] = rec
        del m, x, y
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
