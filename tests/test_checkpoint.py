"""PL-checkpoint loading: a Lightning-format checkpoint of the reference
LitGINI (state_dict + hyper_parameters, with the reference's nn.SiLU activation object among
them, deepinteract_modules.py:1481) is read with torch.load(weights_only=True) only, its
architecture inferred and its keys checked strictly. No trained checkpoint exists offline
(Zenodo), so the files here are written from the seeded reference-keyed state dict."""
import argparse
import os

import pytest
import torch

from deepinteract_amd.weights import check_state_dict, infer_config, read_checkpoint, seeded_state_dict


def _write_ckpt(path, sd, **extra_hp):
    hp = {"num_node_input_feats": 113, "num_edge_input_feats": 27, "gnn_activ_fn": torch.nn.SiLU(),
          "num_gnn_layers": 2, "num_gnn_hidden_channels": 128, "num_gnn_attention_heads": 4, "knn": 20,
          "num_interact_layers": 14, "num_interact_hidden_channels": 128, "lr": 1e-3, "use_wandb_logger": True}
    hp.update(extra_hp)
    torch.save({"epoch": 3, "global_step": 100, "pytorch-lightning_version": "1.4.8",
                "state_dict": sd, "hyper_parameters": hp}, path)


def test_read_lightning_checkpoint_weights_only(tmp_path):
    sd = seeded_state_dict(0)
    p = os.path.join(tmp_path, "LitGINI-GeoTran.ckpt")
    _write_ckpt(p, sd)
    got, arch = read_checkpoint(p)
    assert list(got) == list(sd)
    assert all(torch.equal(got[k], sd[k]) for k in sd)
    assert arch["num_gnn_layers"] == 2 and arch["knn"] == 20 and "lr" not in arch
    cfg = infer_config(got, **arch)
    assert (cfg.num_gnn_layers, cfg.num_gnn_hidden_channels, cfg.num_interact_layers) == (2, 128, 14)
    assert check_state_dict(got, cfg) == []


def test_bare_state_dict_and_shape_inference(tmp_path):
    sd = seeded_state_dict(0)
    p = os.path.join(tmp_path, "sd.pt")
    torch.save(sd, p)
    got, arch = read_checkpoint(p)
    assert arch == {}
    cfg = infer_config(got)
    assert cfg.num_node_input_feats == 113 and cfg.num_gnn_layers == 2 and cfg.num_interact_layers == 14


def test_strict_key_check_reports_problems():
    sd = seeded_state_dict(0)
    cfg = infer_config(sd)
    bad = dict(sd)
    bad.pop("gnn_module.0.gt_block.0.mha_module.Q.weight")
    bad["interact_module.conv2d_1.bias"] = torch.zeros(3)
    probs = check_state_dict(bad, cfg)
    assert any(s.startswith("missing gnn_module.0.gt_block.0.mha_module.Q") for s in probs)
    assert any(s.startswith("shape interact_module.conv2d_1.bias") for s in probs)


def test_checkpoint_needing_other_globals_is_refused(tmp_path):
    """A file whose unpickling needs a global outside the allow-list is never executed."""
    p = os.path.join(tmp_path, "ns.ckpt")
    _write_ckpt(p, seeded_state_dict(0, with_head=False), args=argparse.Namespace(lr=1e-3))
    with pytest.raises(Exception):
        read_checkpoint(p)
    sd, _ = read_checkpoint(p, safe_globals=[argparse.Namespace])  # explicitly allowed by the caller
    assert "node_in_embedding.weight" in sd
