"""Module-at-a-time drop-ins (deepinteract_amd/layers.py) against the CPU oracle's restatement of
the same reference modules, on the tiny golden case's graph (the oracle itself is pinned to the
reference's modules by tests/test_oracle_golden.py). Inputs beyond the fixture (current node /
edge features) are seeded random tensors; weights are the seeded reference-keyed state dict,
sliced to each module's own keys. fp32 <= 1e-4 relative; bf16 bound stated below (measured errors
printed with -s)."""
import numpy as np
import pytest
import torch

from gpu_common import load_case, rel_max
from oracle import geot_oracle as O

pytestmark = pytest.mark.gpu
# bf16 measured on MI355X: init_edge 4.3e-3, conformation 5.7e-3, mha 8.1e-3,
# gt layer 5.2e-3, final 5.4e-3 (max-abs error / max-abs reference); bound ~2x the largest
TOL = {"f32": 1e-4, "bf16": 1.6e-2}


def check(what, dtype, out, ref):
    err = rel_max(_np(out), _np(ref))
    print(f"{what} {dtype}: {err:.3e}")
    assert err < TOL[dtype], (what, dtype, err)
P = "gnn_module.0.gt_block.0"


@pytest.fixture(scope="module")
def sd():
    from deepinteract_amd.weights import seeded_state_dict
    return seeded_state_dict(0)


def sub(sd, pre):
    return {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}


@pytest.fixture(scope="module")
def case():
    from deepinteract_amd.graph import ResidueGraph
    z = load_case("tiny")
    n = int(z["g1_node_f"].shape[0])
    g = ResidueGraph(z["g1_src"], z["g1_dst"], n)
    g.edata["src_nbr_e_ids"] = torch.as_tensor(z["g1_src_nbr"]).long()
    g.edata["dst_nbr_e_ids"] = torch.as_tensor(z["g1_dst_nbr"]).long()
    og = {"num_nodes": n, "src": g.edges()[0], "dst": g.edges()[1], "src_nbr": g.edata["src_nbr_e_ids"],
          "dst_nbr": g.edata["dst_nbr_e_ids"]}
    gen = torch.Generator().manual_seed(7)
    node = torch.randn(n, 128, generator=gen)
    edge = torch.randn(g.num_edges(), 128, generator=gen)
    G = torch.as_tensor(z["g1_edge_f"])
    return g, og, node, edge, G


def _np(t):
    return t.detach().float().cpu().numpy()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_init_edge_module(sd, case, dtype):
    from deepinteract_amd.layers import InitEdgeModule
    g, og, _, _, G = case
    g.edata["f"] = G
    m = InitEdgeModule(dtype).load_reference_state_dict(sub(sd, "gnn_module.0.init_edge_module."))
    out = m(g)
    ref = O.init_edge(sd, og, G)
    check("init_edge", dtype, out, ref)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_conformation_module(sd, case, dtype):
    from deepinteract_amd.layers import ConformationModule
    g, og, _, edge, G = case
    g.edata["f"] = edge
    m = ConformationModule(dtype).load_reference_state_dict(sub(sd, f"{P}.conformation_module."))
    out = m(g, G)
    ref = O.conformation(sd, f"{P}.conformation_module", og, edge, G)
    check("conformation", dtype, out, ref)


@pytest.mark.parametrize("update_edge_feats", [True, False])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_mha_layer(sd, case, dtype, update_edge_feats):
    from deepinteract_amd.layers import MultiHeadGeometricAttentionLayer
    g, og, node, edge, _ = case
    m = MultiHeadGeometricAttentionLayer(128, 32, 4, False, update_edge_feats, dtype=dtype)
    m.load_reference_state_dict(sub(sd, f"{P}.mha_module."))
    h, e = m(g, node, edge)
    rh, re = O.mha(sd, f"{P}.mha_module", og, node, edge, update_edge_feats)
    assert h.shape == (node.shape[0], 4, 32)
    check("mha node", dtype, h, rh)
    if update_edge_feats:
        assert e.shape == (edge.shape[0], 4, 32)
        check("mha edge", dtype, e, re)
    else:
        assert e is None


@pytest.mark.parametrize("final", [False, True])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_geometric_transformer_module(sd, case, dtype, final):
    from deepinteract_amd.layers import FinalGeometricTransformerModule, GeometricTransformerModule
    g, og, node, edge, G = case
    li = 1 if final else 0
    g.ndata["f"], g.edata["f"] = node, edge
    cls = FinalGeometricTransformerModule if final else GeometricTransformerModule
    m = cls(dtype).load_reference_state_dict(sub(sd, f"gnn_module.0.gt_block.{li}."))
    out = m(g, G)
    rn, re, _ = O.gt_layer(sd, li, og, node, edge, G, final)
    if final:
        check("final gt node", dtype, out, rn)
    else:
        n, e = out
        check("gt node", dtype, n, rn)
        check("gt edge", dtype, e, re)


def test_gemm_bias_act_matches_torch():
    """di_gemm_bias_act alone: odd shapes (in 113 -> padded, out 48), bias, SiLU, residual."""
    from deepinteract_amd.layers import _Base
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(77, 113, generator=gen)
    w = torch.randn(48, 113, generator=gen) / 10
    b = torch.randn(48, generator=gen)
    r = torch.randn(77, 48, generator=gen)
    m = _Base("f32")
    m._dev_lin("t", w.double().numpy(), b.double().numpy())
    y = m._gemm("t", x, act=1, res=r)
    ref = torch.nn.functional.silu(x @ w.T + b) + r
    assert rel_max(_np(y), _np(ref)) < 1e-5
