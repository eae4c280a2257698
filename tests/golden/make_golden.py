"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own Python code.

Runs only in the build container (needs /root/reference). The reference's modules execute
unmodified: ``convert_df_to_dgl_graph`` (deepinteract_utils.py:386-555) builds each chain's
graph and ``LitGINI.shared_step`` (deepinteract_modules.py:1687-1745) runs the GeoT +
pair tensor + dilated-ResNet head. Only DGL 0.6 (absent third-party dependency) is
restated, in ``refshim.py``.

Weights: ``deepinteract_amd.weights.seeded_state_dict(0)`` loaded with ``load_state_dict``
(its SHA-256 is stored in every fixture so drift is caught).

Cases (BASELINE.json configs):
  tiny  : synthetic heterodimer 2x48, all intermediates stored in full
  c1    : bundled 4HEQ (project/test_data/4heq_{l,r}_u.pdb), 2x145
  c2    : synthetic homodimer 2x256
  knn1k : kNN indices + squared distances of a 1000-residue synthetic chain (C3 size)

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pandas as pd
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import refshim  # noqa: E402
from deepinteract_amd import synth  # noqa: E402
from deepinteract_amd.weights import seeded_state_dict, state_dict_sha256  # noqa: E402

WEIGHT_SEED = 0
KNN, NB = 20, 2


def chain_to_df(chain):
    """A DIPS-Plus-shaped residue DataFrame (rows N, CA, C, O per residue) for the
    reference's convert_df_to_dgl_graph."""
    bb, am, dips = chain["backbone"], chain["amide_norm"], chain["dips"].astype(np.float64)
    rows = []
    n = bb.shape[0]
    for i in range(n):
        feats = {
            "resname": synth.RESNAMES[int(np.argmax(dips[i, 0:20]))],
            "ss_value": synth.SS_VALUES[int(np.argmax(dips[i, 20:28]))],
            "rsa_value": dips[i, 28], "rd_value": dips[i, 29],
        }
        for j, col in enumerate(['avg_cx', 's_avg_cx', 's_ch_avg_cx', 's_ch_s_avg_cx', 'max_cx', 'min_cx']):
            feats[col] = dips[i, 30 + j]
        feats["hsaac"] = list(dips[i, 36:78])
        feats["cn_value"] = dips[i, 78]
        feats["sequence_feats"] = list(dips[i, 79:106])
        feats["amide_norm_vec"] = am[i].astype(np.float64)
        for a, name in enumerate(("N", "CA", "C", "O")):
            row = {"atom_name": name, "x": float(bb[i, a, 0]), "y": float(bb[i, a, 1]),
                   "z": float(bb[i, a, 2]), "chain": "A", "residue": str(i), "aid": 4 * i + a}
            row.update(feats)
            rows.append(row)
    return pd.DataFrame(rows)


def ref_graph(du, chain, seed):
    df = chain_to_df(chain)
    torch.manual_seed(seed)
    return du.convert_df_to_dgl_graph(df, "synthetic", KNN, NB, True)


def build_model(dm):
    import torch.nn as nn
    m = dm.LitGINI(num_node_input_feats=113, num_edge_input_feats=27, gnn_activ_fn=nn.SiLU(),
                   num_classes=2, num_gnn_layers=2, num_interact_layers=14, dropout_rate=0.2,
                   use_wandb_logger=False)
    sd = seeded_state_dict(WEIGHT_SEED)
    m.load_state_dict(sd)
    m.eval()
    return m, state_dict_sha256(sd)


def run_case(dm, du, model, sha, ch1, ch2, seeds, full: bool, sample_every: int = 1):
    dgl = sys.modules["dgl"]
    g1 = ref_graph(du, ch1, seeds[0])
    g2 = ref_graph(du, ch2, seeds[1])
    out = {"weights_sha256": np.array(sha)}
    for tag, g, ch in (("g1", g1, ch1), ("g2", g2, ch2)):
        src, dst = g.edges()
        out[f"{tag}_backbone"] = ch["backbone"]
        out[f"{tag}_amide_norm"] = ch["amide_norm"]
        out[f"{tag}_dips"] = ch["dips"]
        out[f"{tag}_src"] = src.numpy().astype(np.int32)
        out[f"{tag}_dst"] = dst.numpy().astype(np.int32)
        out[f"{tag}_node_f"] = g.ndata["f"].numpy().astype(np.float32)
        out[f"{tag}_edge_f"] = g.edata["f"].numpy().astype(np.float32)
        out[f"{tag}_src_nbr"] = g.edata["src_nbr_e_ids"].numpy().astype(np.int32)
        out[f"{tag}_dst_nbr"] = g.edata["dst_nbr_e_ids"].numpy().astype(np.int32)
        out[f"{tag}_nbr_seed"] = np.array(seeds[0] if tag == "g1" else seeds[1])
        ca = torch.as_tensor(ch["backbone"][:, 1, :])
        d = sys.modules["dgl.nn.pytorch"].pairwise_squared_distance(ca)
        vals = torch.topk(d, KNN, 1, largest=False).values  # graph_utils.py:108
        out[f"{tag}_d2"] = vals.numpy().astype(np.float32)

    # hooks for intermediates
    rec = {}

    def hook(name):
        def fn(mod, inp, outp):
            rec.setdefault(name, []).append(outp)
        return fn

    gm = model.gnn_module[0]
    hs = [model.node_in_embedding.register_forward_hook(hook("node_emb")),
          gm.init_edge_module.register_forward_hook(hook("init_edge")),
          gm.gt_block[0].conformation_module.register_forward_hook(hook("conf0")),
          gm.gt_block[0].register_forward_hook(hook("layer0")),
          gm.gt_block[1].conformation_module.register_forward_hook(hook("conf1"))]
    with torch.no_grad():
        bg1, bg2 = dgl.batch([g1]), dgl.batch([g2])  # dgl_picp_collate, batch_size=1
        logits_list, n1, e1, n2, e2 = model.shared_step(bg1, bg2, return_representations=True)
        t = du.construct_interact_tensor(torch.as_tensor(n1), torch.as_tensor(n2))
    for h in hs:
        h.remove()
    logits = logits_list[0]
    L1, L2 = logits.shape[-2:]
    flat = torch.flatten(logits.squeeze(0), start_dim=1).transpose(1, 0)  # lit_model_predict.py:236-239
    probs = torch.softmax(flat, dim=1)[:, 1].reshape(L1, L2)
    out["logits"] = logits.numpy().astype(np.float32)
    out["probs"] = probs.numpy().astype(np.float32)
    out["g1_node_out"], out["g2_node_out"] = n1.astype(np.float32), n2.astype(np.float32)
    sel1 = np.arange(0, e1.shape[0], sample_every)
    sel2 = np.arange(0, e2.shape[0], sample_every)
    out["g1_edge_rows"], out["g2_edge_rows"] = sel1.astype(np.int32), sel2.astype(np.int32)
    out["g1_edge_out"], out["g2_edge_out"] = e1[sel1].astype(np.float32), e2[sel2].astype(np.float32)
    out["g1_edge_out_colsum"] = e1.astype(np.float64).sum(0)
    out["g2_edge_out_colsum"] = e2.astype(np.float64).sum(0)
    # pair tensor: checksum + deterministic samples
    t = t.numpy()
    out["pair_shape"] = np.array(t.shape)
    out["pair_sum"] = np.array(t.astype(np.float64).sum())
    rng = np.random.default_rng(7)
    pidx = np.stack([rng.integers(0, s, size=4096) for s in t.shape[1:]], 1)
    out["pair_sample_idx"] = pidx.astype(np.int32)
    out["pair_sample"] = t[0, pidx[:, 0], pidx[:, 1], pidx[:, 2]].astype(np.float32)
    if full:
        for name, vals in rec.items():
            for ci, v in enumerate(vals[:2]):
                tag = f"g{ci + 1}"
                if name == "layer0":
                    out[f"{tag}_layer0_node"] = v[0].numpy().astype(np.float32)
                    out[f"{tag}_layer0_edge"] = v[1].numpy().astype(np.float32)
                else:
                    out[f"{tag}_{name}"] = v.numpy().astype(np.float32)
    return out


def main():
    dm, du = refshim.reference_modules()
    model, sha = build_model(dm)
    print("weights sha256", sha)

    cases = []
    # tiny 2x48 heterodimer, everything stored
    t1, t2 = synth.synthetic_complex(9, 48, 48)
    cases.append(("tiny", t1, t2, (101, 102), True, 1))
    # C1: bundled 4HEQ
    ref_td = os.path.join(refshim.REFERENCE_ROOT, "project", "test_data")
    c1a = synth.read_pdb_chain(os.path.join(ref_td, "4heq_l_u.pdb"), seed=11)
    c1b = synth.read_pdb_chain(os.path.join(ref_td, "4heq_r_u.pdb"), seed=12)
    cases.append(("c1", c1a, c1b, (111, 112), False, 4))
    # C2: synthetic homodimer 2x256
    h1, h2 = synth.synthetic_complex(2, 256, 256, homodimer=True)
    cases.append(("c2", h1, h2, (121, 122), False, 16))

    for name, a, b, seeds, full, every in cases:
        out = run_case(dm, du, model, sha, a, b, seeds, full, every)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **out)
        print(name, path, os.path.getsize(path) // 1024, "KiB", out["logits"].shape)

    # kNN at C3 size (graph_utils.py:107-108 through the DGL restatement)
    ch = synth.synthetic_chain(1000, 10_000 * 3 + 1)
    ca = torch.as_tensor(ch["backbone"][:, 1, :])
    g = sys.modules["dgl"].knn_graph(ca, KNN)
    d = sys.modules["dgl.nn.pytorch"].pairwise_squared_distance(ca)
    vals = torch.topk(d, KNN, 1, largest=False).values
    np.savez_compressed(os.path.join(HERE, "knn1k.npz"), ca=ch["backbone"][:, 1, :],
                        idx=g.edges()[0].numpy().reshape(1000, KNN).astype(np.int32),
                        d2=vals.numpy().astype(np.float32))
    print("knn1k done")


if __name__ == "__main__":
    main()
