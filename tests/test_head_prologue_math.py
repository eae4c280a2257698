"""CPU check of the algebra di_head_prologue relies on, in float64:
conv2d_1 (1x1) on the outer-concat pair tensor separates per chain, and InstanceNorm2d's
statistics of the separable sum are the sums of the per-chain means and biased variances. The
restatement below is the kernel's dataflow (k_prologue_tables + k_prologue_rows); the reference
side is the oracle's op-for-op ELU(inorm_1(conv2d_1(T))) on the materialised T."""
import numpy as np
import torch

from oracle import geot_oracle as O


def fused_prologue(h1, h2, w, b, gamma, beta, eps):
    H = h1.shape[1]
    A = h1 @ w[:, :H].T                     # [L1, C]
    B = h2 @ w[:, H:].T + b                 # [L2, C]
    ma, mb = A.mean(0), B.mean(0)
    var = ((A - ma) ** 2).mean(0) + ((B - mb) ** 2).mean(0)
    s = gamma / np.sqrt(var + eps)
    a = s * (A - ma) + beta
    bb = s * (B - mb)
    x = a.T[:, :, None] + bb.T[:, None, :]  # [C, L1, L2]
    return np.where(x > 0, x, np.expm1(x))


def test_separable_conv_and_analytic_instance_norm():
    rng = np.random.default_rng(0)
    L1, L2, H, C = 23, 31, 16, 8
    h1, h2 = rng.normal(size=(L1, H)) * 2, rng.normal(size=(L2, H))
    w = rng.normal(size=(C, 2 * H)) / np.sqrt(2 * H)
    b, gamma, beta = rng.normal(size=C) * 0.1, 1 + 0.2 * rng.normal(size=C), 0.2 * rng.normal(size=C)
    sd = {"interact_module.conv2d_1.weight": torch.tensor(w).reshape(C, 2 * H, 1, 1),
          "interact_module.conv2d_1.bias": torch.tensor(b),
          "interact_module.inorm_1.weight": torch.tensor(gamma),
          "interact_module.inorm_1.bias": torch.tensor(beta)}
    with torch.no_grad():
        ref = O.head_prologue(sd, O.pair_tensor(torch.tensor(h1), torch.tensor(h2)))[0].numpy()
    got = fused_prologue(h1, h2, w, b, gamma, beta, O.IN_EPS)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-10)
