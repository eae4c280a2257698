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


def test_node_count_limit_inferred_from_positional_table():
    from deepinteract_amd.config import GeoTConfig
    sd = seeded_state_dict(0, GeoTConfig(node_count_limit=4096), with_head=False)
    assert infer_config(sd).node_count_limit == 4096
    assert infer_config(seeded_state_dict(0, with_head=False)).node_count_limit == 2304


def test_litgini_rejects_unsupported_heads_and_width():
    from deepinteract_amd.modules import LitGINI
    with pytest.raises(NotImplementedError):
        LitGINI(num_gnn_attention_heads=8)
    with pytest.raises(NotImplementedError):
        LitGINI(num_gnn_hidden_channels=64)


def test_litgini_passes_max_num_graph_nodes_to_config():
    from deepinteract_amd.modules import LitGINI
    assert LitGINI(max_num_graph_nodes=4096).cfg.node_count_limit == 4096
    assert LitGINI().cfg.node_count_limit == 2304
    # a checkpoint with a larger positional table loads: the GeoT kernels only need
    # node_pos < max_num_graph_nodes; the on-device builder's 4096-residue chain limit is its own
    assert LitGINI(max_num_graph_nodes=8192).cfg.node_count_limit == 8192
    with pytest.raises(ValueError):
        LitGINI(max_num_graph_nodes=0)


def test_builder_refuses_chains_beyond_the_knn_limit():
    """build_graph_batch raises before touching the device for a chain beyond the kNN's 4096 rows
    (even when the model's positional table is larger)."""
    import numpy as np
    from deepinteract_amd.builder import build_graph_batch
    n = 4097
    ch = {"backbone": np.zeros((n, 4, 3), np.float32), "amide_norm": np.zeros((n, 3), np.float32),
          "dips": np.zeros((n, 106), np.float32)}
    with pytest.raises(NotImplementedError):
        build_graph_batch([ch], node_count_limit=8192, device="cuda")


def test_load_on_cpu_does_not_touch_the_gpu_and_refuses_cpu_compute(tmp_path):
    """load_from_checkpoint without map_location (lit_model_predict.py:214) builds on the CPU; the
    GeoT weights are packed for the GPU only at first use, and a CPU-resident model raises
    rather than handing host pointers to a kernel."""
    from deepinteract_amd.graph import ResidueGraph
    from deepinteract_amd.modules import LitGINI
    sd = seeded_state_dict(0)
    p = os.path.join(tmp_path, "m.ckpt")
    _write_ckpt(p, sd)
    m = LitGINI.load_from_checkpoint(p).freeze()
    assert next(m.parameters()).device.type == "cpu"
    g = ResidueGraph(torch.zeros(40, dtype=torch.long), torch.arange(2).repeat_interleave(20), 2)
    with pytest.raises(RuntimeError):
        m.gnn_forward(g)
