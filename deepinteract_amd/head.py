"""Dilated-ResNet contact head — stays on PyTorch-ROCm (MIOpen convolutions), as north_star
specifies. Module/parameter names match the reference's ``interact_module`` so reference
state dicts load unchanged: ResNet2DInputWithOptAttention (deepinteract_modules.py:1155-1248),
ResNet (:973-1106), SEBlock (:954-970). The optional regional attention (MHA2D) is not part
of the default model (``use_interact_attention=False``) and is not implemented.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class SEBlock(nn.Module):
    def __init__(self, ch, ratio=16):
        super().__init__()
        self.linear1 = nn.Linear(ch, ch // ratio)
        self.linear2 = nn.Linear(ch // ratio, ch)

    def forward(self, x):
        s = x.mean(dim=(2, 3))
        s = torch.sigmoid(F.relu(self.linear2(F.relu(self.linear1(s)))))
        return x * s[:, :, None, None]


class ResNet(nn.Module):
    def __init__(self, num_channels, num_chunks, module_name, inorm=False, initial_projection=False,
                 extra_blocks=False, dilation_cycle=(1, 2, 4, 8)):
        super().__init__()
        self.module_name, self.inorm = module_name, inorm
        self.initial_projection = initial_projection
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
        for r in self.blocks:
            res = x
            for i in (1, 2, 3):
                if self.inorm:
                    x = m[f"{r}_inorm_{i}"](x)
                x = m[f"{r}_conv2d_{i}"](F.elu(x))
            x = m[f"{r}_se_block"](x) + res
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

    def forward(self, t):
        return self.body(F.elu(self.inorm_1(self.conv2d_1(t))))

    def body(self, x):
        """Everything after the prologue ELU(inorm_1(conv2d_1(t))) (which HeadPrologueOp fuses
        with the pair tensor on HIP)."""
        x = F.elu(self.base_resnet(x))
        x = F.elu(self.phase2_resnet(x))
        return self.phase2_conv(x)


def contact_probs(logits):
    """lit_model_predict.py:236-239: softmax over classes, positive class, [L1, L2]."""
    return torch.softmax(logits.squeeze(0), dim=0)[1]
