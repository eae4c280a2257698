"""GPU parity of the head's HIP norm passes (csrc/head_ops.hip, head.HeadNormOps) against plain
PyTorch fp32 on the same inputs: ELU(InstanceNorm2d(x)) (deepinteract_modules.py:1016-1030,
1075-1095) and SEBlock gate + residual (:954-970, :1095).

Tolerances: fp32 ELU(InstanceNorm) <= 2e-6 relative to max |ref| (fp64 statistics vs torch's fp32
Welford: rounding-level); fp32 SE+residual bit-exact (same two roundings as torch); bf16 within two
bf16 ulps of an fp64 evaluation on the same bf16 input, SE+residual bit-exact.
Shapes cover aligned planes (C3's 1000x1000 rows), unaligned planes (145x145: the 4HEQ case) and
planes shorter than one 16-B vector.
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(128, 64, 64), (64, 145, 145), (7, 3, 3), (3, 1, 5), (128, 1000, 1000)]


@pytest.fixture(scope="module")
def ops():
    from deepinteract_amd.head import HeadNormOps
    return HeadNormOps("cuda")


def _norm(C, seed):
    g = torch.Generator().manual_seed(seed)
    m = nn.InstanceNorm2d(C, eps=1e-6, affine=True)
    with torch.no_grad():
        m.weight.copy_(1 + 0.3 * torch.randn(C, generator=g))
        m.bias.copy_(0.3 * torch.randn(C, generator=g))
    return m.cuda()


def _x(C, H, W, seed, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    # per-channel offsets and scales so the statistics are non-trivial
    x = torch.randn(1, C, H, W, generator=g) * (0.5 + torch.rand(C, generator=g))[None, :, None, None] \
        + 3 * torch.randn(C, generator=g)[None, :, None, None]
    return x.cuda().to(dtype)


@pytest.mark.parametrize("shape", SHAPES)
def test_inorm_elu_f32(ops, shape):
    C, H, W = shape
    x, m = _x(C, H, W, 1), _norm(C, 2)
    ref = F.elu(F.instance_norm(x.double(), weight=m.weight.double(), bias=m.bias.double(), eps=m.eps)).float()
    y = ops.inorm_elu(x, m)
    assert float((y - ref).abs().max() / ref.abs().max()) < 2e-6
    x2 = x.clone()
    ops.inorm_elu(x2, m, out=x2)  # in place
    assert torch.equal(x2, y)


@pytest.mark.parametrize("shape", SHAPES[:4])
def test_inorm_elu_bf16(ops, shape):
    C, H, W = shape
    x, m = _x(C, H, W, 3, torch.bfloat16), _norm(C, 4)
    # fp64 reference on the same bf16 input (torch's fp32 GPU instance norm is itself off by a few
    # 1e-4 here: E[x^2] - E[x]^2 accumulated in fp32 over channels with large means)
    ref = F.elu(F.instance_norm(x.double(), weight=m.weight.double(), bias=m.bias.double(), eps=m.eps)).float()
    y = ops.inorm_elu(x, m).float()
    ulp = ref.abs().clamp_min(2 ** -20) * 2 ** -7
    bad = (y - ref).abs() > 2 * ulp + 1e-6
    assert not bool(bad.any()), (f"{int(bad.sum())} elements, e.g. y={y[bad][:4].tolist()} "
                                 f"ref={ref[bad][:4].tolist()}")


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_se_scale_add_exact(ops, shape, dtype):
    C, H, W = shape
    x, res = _x(C, H, W, 5, dtype), _x(C, H, W, 6, dtype)
    s = torch.sigmoid(torch.randn(1, C, generator=torch.Generator().manual_seed(7))).cuda().to(dtype)
    ref = x * s[:, :, None, None] + res
    y = ops.se_scale_add(x, s, res)
    assert torch.equal(y, ref)
    # with the deferred conv bias: torch's order is (x + b) -> * s -> + res, each rounded
    b = torch.randn(C, generator=torch.Generator().manual_seed(8)).cuda()
    xb = x + b.to(dtype)[None, :, None, None] if dtype == torch.bfloat16 else x + b[None, :, None, None]
    ref_b = xb * s[:, :, None, None] + res
    assert torch.equal(ops.se_scale_add(x, s, res, bias=b.to(dtype)), ref_b)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_channel_mean(ops, shape, dtype):
    C, H, W = shape
    x = _x(C, H, W, 9, dtype)
    b = torch.randn(C, generator=torch.Generator().manual_seed(10)).cuda()
    ref = x.double().mean(dim=(2, 3)) + b.double()[None]
    m = ops.channel_mean(x, b)
    assert float((m.double() - ref).abs().max()) < 1e-6 * float(ref.abs().max()) + 1e-7


def test_head_body_with_hip_ops_matches_torch_f32():
    """The whole head (58 ResNet blocks) with the HIP passes (bias folding, SE fusion) vs torch's
    passes, fp32, 64x64."""
    from deepinteract_amd.head import HeadNormOps, ResNet2DInputWithOptAttention
    from deepinteract_amd.weights import seeded_state_dict
    sd = seeded_state_dict(0)
    hsd = {k[len("interact_module."):]: v for k, v in sd.items() if k.startswith("interact_module.")}
    a = ResNet2DInputWithOptAttention().cuda().eval()
    a.load_state_dict(hsd)
    b = ResNet2DInputWithOptAttention().cuda().eval()
    b.load_state_dict(hsd)
    b.use_hip_norm_ops(HeadNormOps("cuda"))
    t = torch.randn(1, 256, 64, 64, generator=torch.Generator().manual_seed(0)).cuda()
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=False):
        ya, yb = a(t), b(t)
    assert float((ya - yb).abs().max() / ya.abs().max()) < 1e-5
