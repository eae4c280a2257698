"""the reference's parameter initialisation (glorot_orthogonal,
deepinteract_utils.py:47-52, and each module's reset_parameters), restated in
weights.reference_init_state_dict. CPU only."""
import math

import torch

from deepinteract_amd.config import GeoTConfig
from deepinteract_amd.weights import (check_state_dict, glorot_orthogonal, reference_init_state_dict,
                                      seeded_state_dict)


def test_glorot_orthogonal_semantics():
    g = torch.Generator().manual_seed(0)
    for shape in [(128, 128), (64, 128), (128, 256), (28, 128), (128, 18)]:
        w = glorot_orthogonal(torch.empty(shape), 2.0, generator=g)
        # var(W) * (fan_out + fan_in) == scale after the rescale
        assert abs(float(w.var()) * (shape[0] + shape[1]) - 2.0) < 1e-4
        # the orthogonal_ structure survives the scalar rescale
        q = w @ w.T if shape[0] <= shape[1] else w.T @ w
        d = torch.diagonal(q)
        assert torch.allclose(q, torch.diag(d), atol=1e-5 * float(d.max()))
        assert torch.allclose(d, d[0].expand_as(d), rtol=1e-4)


def test_reference_init_state_dict_matches_reset_parameters():
    cfg = GeoTConfig()
    sd = reference_init_state_dict(0, cfg)
    assert check_state_dict(sd, cfg) == []
    assert set(sd) == set(seeded_state_dict(0, cfg))
    p = "gnn_module.0.gt_block.0.conformation_module"
    assert float(sd[f"{p}.nbr_linear.bias"].abs().max()) == 0.0  # fill_(0), :354
    w = sd[f"{p}.nbr_linear.weight"]
    assert abs(float(w.var()) * (w.shape[0] + w.shape[1]) - 2.0) < 1e-4
    emb = sd["gnn_module.0.init_edge_module.node_embedding.weight"]
    assert float(emb.abs().max()) <= math.sqrt(3.0)
    # the one BatchNorm of a ResBlock, registered at .1/.4/.7, holds one set of values
    rb = [k for k in sd if ".res_block.1.running_var" in k][0]
    assert torch.equal(sd[rb], sd[rb.replace(".res_block.1.", ".res_block.4.")])
    assert float(sd[rb].min()) == 1.0
    b = sd["interact_module.phase2_conv.bias"]
    assert float(b[1]) == -7.0 and abs(float(b[0])) <= 1.0 / math.sqrt(128)  # :1224-1226
    c = sd["interact_module.base_resnet.resnet_base_resnet_0_1_conv2d_2.weight"]
    assert float(c.abs().max()) <= 1.0 / math.sqrt(64 * 9)
    assert torch.equal(reference_init_state_dict(0, cfg)[f"{p}.nbr_linear.weight"], w)  # seeded
