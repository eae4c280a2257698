"""Dilated-ResNet contact head — stays on PyTorch-ROCm (MIOpen convolutions), as north_star
specifies. Module/parameter names match the reference's ``interact_module`` so reference
state dicts load unchanged: ResNet2DInputWithOptAttention (deepinteract_modules.py:1155-1248),
ResNet (:973-1106), SEBlock (:954-970). The optional regional attention (MHA2D) is not part
of the default model (``use_interact_attention=False``) and is not implemented.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F


class HeadNormOps:
    """The head's HBM-bound passes on HIP (csrc/head_ops.hip): ELU(InstanceNorm2d(x))
    in 3 plane passes instead of torch's 5, and SEBlock gate + residual add in 3 instead of 5.
    Inputs: one [1, C, H, W] NCHW-contiguous image, fp32 or bf16, on the GPU. No CPU fallback:
    constructing it without the HIP library / a GPU raises."""

    def __init__(self, device):
        from . import _lib
        if not torch.cuda.is_available():
            raise RuntimeError("HeadNormOps needs a ROCm GPU (no CPU fallback)")
        self._lib = _lib
        self.lib = _lib.load()
        self.device = torch.device(device)
        self._work = None
        self._f32 = {}  # fp32 copies of (bf16) per-channel parameters, made once per parameter

    def f32(self, p):
        """fp32 contiguous copy of a (possibly bf16) per-channel parameter, cached."""
        if p is None:
            return None
        hit = self._f32.get(id(p))
        # the entry holds p itself, so its id cannot be reused by another tensor while cached
        if hit is None or hit[0] is not p or hit[1] != p._version:
            hit = self._f32[id(p)] = (p, p._version, p.detach().float().contiguous())
        return hit[2]

    def work(self, C, hw, device):
        nb = self.lib.di_inorm_work_bytes(C, hw)
        if self._work is None or self._work.numel() * 8 < nb:
            self._work = torch.empty((nb + 7) // 8, dtype=torch.float64, device=device)
        return self._work

    def _dt(self, x):
        if x.dtype == torch.float32:
            return self._lib.DI_F32
        if x.dtype == torch.bfloat16:
            return self._lib.DI_BF16
        raise TypeError(f"head ops take fp32 / bf16, got {x.dtype}")

    @staticmethod
    def _check(x):
        if x.dim() != 4 or x.shape[0] != 1 or not x.is_contiguous() or not x.is_cuda:
            raise ValueError("head ops take one contiguous NCHW [1, C, H, W] GPU image")

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def inorm_elu(self, x, norm: nn.InstanceNorm2d, out=None):
        """F.elu(norm(x)); out may be x (in place)."""
        self._check(x)
        C, hw = x.shape[1], x.shape[2] * x.shape[3]
        y = torch.empty_like(x) if out is None else out
        w = self.work(C, hw, x.device)
        g, b = self.f32(norm.weight), self.f32(norm.bias)
        self._lib.check(self.lib.di_inorm_elu(self._dt(x), ctypes.c_void_p(x.data_ptr()), C, hw,
                                              ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                              ctypes.c_float(norm.eps), ctypes.c_void_p(w.data_ptr()),
                                              ctypes.c_void_p(y.data_ptr()), self._stream()), "di_inorm_elu")
        return y

    def channel_mean(self, x, bias=None):
        """x.mean(dim=(2, 3)) (+ bias) as fp32 [1, C]."""
        self._check(x)
        C, hw = x.shape[1], x.shape[2] * x.shape[3]
        w = self.work(C, hw, x.device)
        m = torch.empty(1, C, dtype=torch.float32, device=x.device)
        b = self.f32(bias)
        self._lib.check(self.lib.di_channel_mean(self._dt(x), ctypes.c_void_p(x.data_ptr()), C, hw,
                                                 ctypes.c_void_p(0 if b is None else b.data_ptr()),
                                                 ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(m.data_ptr()),
                                                 self._stream()), "di_channel_mean")
        return m

    def se_scale_add(self, x, scale, res, out=None, bias=None):
        """(x + bias[None, :, None, None]) * scale[None, :, None, None] + res; out may be x or res."""
        self._check(x)
        self._check(res)
        C, hw = x.shape[1], x.shape[2] * x.shape[3]
        s = scale.detach().reshape(-1).float().contiguous()
        b = self.f32(bias)
        y = torch.empty_like(x) if out is None else out
        self._lib.check(self.lib.di_se_scale_add(self._dt(x), ctypes.c_void_p(x.data_ptr()),
                                                 ctypes.c_void_p(s.data_ptr()),
                                                 ctypes.c_void_p(0 if b is None else b.data_ptr()),
                                                 ctypes.c_void_p(res.data_ptr()), C, hw,
                                                 ctypes.c_void_p(y.data_ptr()), self._stream()),
                        "di_se_scale_add")
        return y


class SEBlock(nn.Module):
    def __init__(self, ch, ratio=16):
        super().__init__()
        self.linear1 = nn.Linear(ch, ch // ratio)
        self.linear2 = nn.Linear(ch // ratio, ch)

    def gate(self, x):
        return self.gate_from_mean(x.mean(dim=(2, 3)))

    def gate_from_mean(self, s):
        s = s.to(self.linear1.weight.dtype)
        return torch.sigmoid(F.relu(self.linear2(F.relu(self.linear1(s)))))

    def forward(self, x):
        return x * self.gate(x)[:, :, None, None]


class ResNet(nn.Module):
    def __init__(self, num_channels, num_chunks, module_name, inorm=False, initial_projection=False,
                 extra_blocks=False, dilation_cycle=(1, 2, 4, 8)):
        super().__init__()
        self.module_name, self.inorm = module_name, inorm
        self.initial_projection = initial_projection
        self.ops = None  # HeadNormOps: fused norm/ELU and SE/residual passes on HIP
        C = num_channels
        self.blocks = []
        if initial_projection:
            self.add_module(f"resnet_{module_name}_init_proj", nn.Conv2d(C, C, 1))
        names = [(f"{i}_{d}", d) for i in range(num_chunks) for d in dilation_cycle]
        if extra_blocks:
            names += [("extra0", 1), ("extra1", 1)]
        for b, d in names:
            r = f"resnet_{module_name}_{b}"
            if inorm:
                self.add_module(f"{r}_inorm_1", nn.InstanceNorm2d(C, eps=1e-06, affine=True))
                self.add_module(f"{r}_inorm_2", nn.InstanceNorm2d(C // 2, eps=1e-06, affine=True))
                self.add_module(f"{r}_inorm_3", nn.InstanceNorm2d(C // 2, eps=1e-06, affine=True))
            self.add_module(f"{r}_conv2d_1", nn.Conv2d(C, C // 2, 1))
            self.add_module(f"{r}_conv2d_2", nn.Conv2d(C // 2, C // 2, 3, dilation=d, padding=d))
            self.add_module(f"{r}_conv2d_3", nn.Conv2d(C // 2, C, 1))
            self.add_module(f"{r}_se_block", SEBlock(C, 16))
            self.blocks.append(r)

    def forward(self, x):
        m = self._modules
        if self.initial_projection:
            x = m[f"resnet_{self.module_name}_init_proj"](x)
        ops = self.ops
        if ops is not None:
            return self._forward_hip(x, ops)
        for r in self.blocks:
            res = x
            for i in (1, 2, 3):
                if self.inorm:
                    x = m[f"{r}_inorm_{i}"](x)
                x = m[f"{r}_conv2d_{i}"](F.elu(x))
            x = m[f"{r}_se_block"](x) + res
        return x

    def _forward_hip(self, x, ops):
        """Same blocks with the norm / bias / SE passes on HIP (HeadNormOps). A conv that feeds an
        InstanceNorm runs without its bias (a per-channel constant cancels in the normalisation);
        the last conv's bias is applied inside the SE gate + residual pass, and the SE squeeze
        (channel mean) adds it analytically."""
        m = self._modules
        for r in self.blocks:
            res = x
            for i in (1, 2, 3):
                conv = m[f"{r}_conv2d_{i}"]
                if self.inorm:
                    x = ops.inorm_elu(x, m[f"{r}_inorm_{i}"], out=None if i == 1 else x)
                else:
                    x = F.elu(x)
                keep_bias = not self.inorm and i < 3
                x = F.conv2d(x, conv.weight, conv.bias if keep_bias else None, conv.stride, conv.padding,
                             conv.dilation)
            conv3, se = m[f"{r}_conv2d_3"], m[f"{r}_se_block"]
            gate = se.gate_from_mean(ops.channel_mean(x, conv3.bias))
            x = ops.se_scale_add(x, gate, res, out=x, bias=conv3.bias)
        return x


class ResNet2DInputWithOptAttention(nn.Module):
    def __init__(self, num_chunks=14, init_channels=256, num_channels=128, num_classes=2):
        super().__init__()
        self.conv2d_1 = nn.Conv2d(init_channels, num_channels, 1)
        self.inorm_1 = nn.InstanceNorm2d(num_channels, eps=1e-06, affine=True)
        self.base_resnet = ResNet(num_channels, num_chunks, "base_resnet", inorm=True, initial_projection=True)
        self.phase2_resnet = ResNet(num_channels, 1, "bin_resnet", inorm=False, initial_projection=True,
                                    extra_blocks=True)
        self.phase2_conv = nn.Conv2d(num_channels, num_classes, 1)
        self.ops = None

    def use_hip_norm_ops(self, ops):
        """Route the InstanceNorm+ELU and SE+residual passes through HeadNormOps (or None: torch)."""
        self.ops = self.base_resnet.ops = self.phase2_resnet.ops = ops
        return self

    def forward(self, t):
        x = self.conv2d_1(t)
        if getattr(self, "ops", None) is not None:
            return self.body(self.ops.inorm_elu(x, self.inorm_1, out=x))
        return self.body(F.elu(self.inorm_1(x)))

    def body(self, x):
        """Everything after the prologue ELU(inorm_1(conv2d_1(t))) (which HeadPrologueOp fuses
        with the pair tensor on HIP)."""
        x = F.elu(self.base_resnet(x))
        x = F.elu(self.phase2_resnet(x))
        return self.phase2_conv(x)


def contact_probs(logits):
    """lit_model_predict.py:236-239: softmax over classes, positive class, [L1, L2]."""
    return torch.softmax(logits.squeeze(0), dim=0)[1]
