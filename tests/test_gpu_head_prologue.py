"""GPU parity of the fused head prologue (di_head_prologue):
ELU(inorm_1(conv2d_1(T))) computed from the node features without materialising the pair
tensor T, against the oracle's op-for-op restatement on the materialised T
(oracle.geot_oracle.head_prologue, deepinteract_modules.py:1231-1232).

Tolerances: fp32 output <= 1e-4 relative (max-abs error / max-abs reference); bf16 output
(bf16 node features in, fp32 statistics, bf16 store) <= 1e-2 relative against the fp32 reference
evaluated on the same bf16-rounded node features. End to end: LitGINI(fuse_head_prologue=True)
logits and contact probabilities within 1e-4 of the golden vectors made by the reference's code.
"""
import numpy as np
import pytest
import torch

from gpu_common import chain_item, load_case, rel_max

pytestmark = pytest.mark.gpu


def _head_params(seed, C=128, H=128):
    g = torch.Generator().manual_seed(seed)
    return {
        "interact_module.conv2d_1.weight": torch.randn(C, 2 * H, 1, 1, generator=g) / np.sqrt(2 * H),
        "interact_module.conv2d_1.bias": torch.randn(C, generator=g) * 0.1,
        "interact_module.inorm_1.weight": 1 + 0.2 * torch.randn(C, generator=g),
        "interact_module.inorm_1.bias": 0.2 * torch.randn(C, generator=g),
    }


@pytest.mark.parametrize("dtype,sizes", [
    (torch.float32, [(40, 36), (264, 100)]),        # aligned (L2 % 4 == 0): row-streaming stores
    (torch.float32, [(37, 45), (9, 130)]),          # unaligned: flat kernel
    (torch.bfloat16, [(48, 64), (300, 1000)]),      # aligned (L2 % 8 == 0), several row blocks
    (torch.bfloat16, [(13, 21)]),                   # unaligned
])
def test_head_prologue_matches_oracle(dtype, sizes):
    from deepinteract_amd.engine import HeadPrologueOp
    from oracle import geot_oracle as O
    torch.manual_seed(3)
    sd = _head_params(5)
    rows = sum(a + b for a, b in sizes)
    h = (torch.randn(rows, 128) * 2).to(dtype)
    op = HeadPrologueOp(sd["interact_module.conv2d_1.weight"], sd["interact_module.conv2d_1.bias"],
                        sd["interact_module.inorm_1.weight"], sd["interact_module.inorm_1.bias"], 1e-6, "cuda")
    h1r, h2r, r = [], [], 0
    for a, b in sizes:
        h1r.append(r)
        h2r.append(r + a)
        r += a + b
    _, views = op(h.cuda(), h1r, h2r, [a for a, _ in sizes], [b for _, b in sizes])
    torch.cuda.synchronize()
    hf = h.float()
    tol = 1e-4 if dtype == torch.float32 else 1e-2
    for (a, b), s1, s2, v in zip(sizes, h1r, h2r, views):
        with torch.no_grad():
            ref = O.head_prologue(sd, O.pair_tensor(hf[s1:s1 + a], hf[s2:s2 + b]))
        assert v.shape == ref.shape
        assert rel_max(v.float().cpu().numpy(), ref.numpy()) < tol


@pytest.mark.parametrize("C,H,sizes", [
    (40, 64, [(70, 36), (4200, 12)]),   # channels % 16 != 0; 66 row tiles on one side (> one wave)
    (13, 128, [(65, 128), (1, 8)]),     # fewer channels than one table block; single-row chain
])
def test_head_prologue_ragged_channels_and_many_tiles(C, H, sizes):
    """The table kernels split rows into 64-row tiles and channels into groups of 16; the
    per-channel statistics are merged from the tile summaries (fp32, <= 1e-4)."""
    from deepinteract_amd.engine import HeadPrologueOp
    from oracle import geot_oracle as O
    torch.manual_seed(7)
    sd = _head_params(8, C=C, H=H)
    rows = sum(a + b for a, b in sizes)
    h = torch.randn(rows, H) * 2
    op = HeadPrologueOp(sd["interact_module.conv2d_1.weight"], sd["interact_module.conv2d_1.bias"],
                        sd["interact_module.inorm_1.weight"], sd["interact_module.inorm_1.bias"], 1e-6, "cuda")
    h1r, h2r, r = [], [], 0
    for a, b in sizes:
        h1r.append(r)
        h2r.append(r + a)
        r += a + b
    _, views = op(h.cuda(), h1r, h2r, [a for a, _ in sizes], [b for _, b in sizes])
    torch.cuda.synchronize()
    for (a, b), s1, s2, v in zip(sizes, h1r, h2r, views):
        with torch.no_grad():
            ref = O.head_prologue(sd, O.pair_tensor(h[s1:s1 + a], h[s2:s2 + b]))
        assert v.shape == ref.shape
        assert rel_max(v.float().cpu().numpy(), ref.numpy()) < 1e-4


def test_head_prologue_bf16_wide_range_channels_take_exact_exp():
    """Channels whose folded tables exceed |60| (gamma x 200) leave the e^a e^b product path for
    the exact exp path; results stay within the bf16 tolerance on every channel."""
    from deepinteract_amd.engine import HeadPrologueOp
    from oracle import geot_oracle as O
    torch.manual_seed(4)
    sd = _head_params(6)
    sd["interact_module.inorm_1.weight"][::2] *= 200.0
    a, b = 64, 128
    h = (torch.randn(a + b, 128) * 2).to(torch.bfloat16)
    op = HeadPrologueOp(sd["interact_module.conv2d_1.weight"], sd["interact_module.conv2d_1.bias"],
                        sd["interact_module.inorm_1.weight"], sd["interact_module.inorm_1.bias"], 1e-6, "cuda")
    _, views = op(h.cuda(), [0], [a], [a], [b])
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = O.head_prologue(sd, O.pair_tensor(h.float()[:a], h.float()[a:]))[0]
    got = views[0][0].float().cpu()
    for c in range(ref.shape[0]):
        assert rel_max(got[c].numpy(), ref[c].numpy()) < 1e-2, c


def test_head_prologue_rejects_bad_shapes():
    from deepinteract_amd.engine import HeadPrologueOp
    sd = _head_params(1, H=64)
    op = HeadPrologueOp(sd["interact_module.conv2d_1.weight"], sd["interact_module.conv2d_1.bias"],
                        sd["interact_module.inorm_1.weight"], sd["interact_module.inorm_1.bias"], 1e-6, "cuda")
    with pytest.raises(ValueError):
        op(torch.randn(10, 128, device="cuda"), [0], [5], [5], [5])  # conv expects 2 x 64 channels


@pytest.mark.parametrize("case", ["tiny", "c1"])
def test_fused_prologue_end_to_end_logits(case):
    """GeoT (HIP) -> fused prologue (HIP) -> head body (torch) == golden logits / probabilities."""
    from deepinteract_amd.graph import GraphBatch
    from deepinteract_amd.modules import LitGINI
    from deepinteract_amd.weights import seeded_state_dict
    z = load_case(case)
    sd = seeded_state_dict(0)
    model = LitGINI(dtype="f32", precise_head=True, fuse_head_prologue=True).cuda().eval()
    model.load_reference_state_dict(sd)
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    with torch.no_grad():
        logits, probs = model.predict_batch(gb, [(0, 1)])
    torch.cuda.synchronize()
    assert rel_max(logits[0].cpu().numpy(), z["logits"]) < 1e-4
    assert rel_max(probs[0].cpu().numpy(), z["probs"]) < 1e-4


def test_load_from_checkpoint_end_to_end_logits(tmp_path):
    """LitGINI.load_from_checkpoint on a Lightning-format file (weights-only read) reproduces the
    golden logits made by the reference's code from the same seeded weights."""
    import os
    from deepinteract_amd.graph import GraphBatch
    from deepinteract_amd.modules import LitGINI
    from deepinteract_amd.weights import seeded_state_dict
    z = load_case("tiny")
    p = os.path.join(tmp_path, "LitGINI.ckpt")
    torch.save({"state_dict": seeded_state_dict(0),
                "hyper_parameters": {"gnn_activ_fn": torch.nn.SiLU(), "num_gnn_layers": 2, "knn": 20}}, p)
    model = LitGINI.load_from_checkpoint(p, map_location="cuda", use_wandb_logger=False, batch_size=1,
                                         precise_head=True).freeze()
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    with torch.no_grad():
        logits, probs = model.predict_batch(gb, [(0, 1)])
    torch.cuda.synchronize()
    assert rel_max(logits[0].cpu().numpy(), z["logits"]) < 1e-4
    assert rel_max(probs[0].cpu().numpy(), z["probs"]) < 1e-4
