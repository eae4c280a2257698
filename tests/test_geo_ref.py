"""DI_GRAPH_GEO_REF (include/deepinteract_amd.h): the reference featuriser's constant direction /
orientation edge columns, and what they make exactly zero or constant in the reference's modules.

CPU checks on the reference-made fixtures (tests/golden, produced by the reference's own
convert_df_to_dgl_graph): the columns are (0,0,0, 0,0,0,1) on every edge; with them the conformation
module's neighbour messages (deepinteract_modules.py:384-418) are exactly zero, InitEdge's direction
terms are exactly zero, and its orientation terms equal the packed constants (packing.init_blob).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from gpu_common import chain_item, load_case

from deepinteract_amd.graph import GEO_REF_COLS, GEO_REF_VALUES, GraphBatch, edge_feats_geo_ref
from deepinteract_amd.packing import GEO_ORDER, init_blob
from deepinteract_amd.weights import seeded_state_dict
from oracle import geot_oracle as O


@pytest.mark.parametrize("case", ["tiny", "c1", "c2"])
def test_reference_featuriser_columns_are_the_constants(case):
    z = load_case(case)
    for tag in ("g1", "g2"):
        ef = torch.as_tensor(z[f"{tag}_edge_f"])
        lo, hi = GEO_REF_COLS
        assert torch.equal(ef[:, lo:hi], torch.tensor(GEO_REF_VALUES).expand(ef.shape[0], hi - lo))
        assert edge_feats_geo_ref(ef)


def test_geo_ref_detection_and_propagation():
    z = load_case("tiny")
    items = [chain_item(z, "g1"), chain_item(z, "g2")]
    gb = GraphBatch.from_arrays(items, "cpu")
    assert gb.geo_ref and gb.c_graph.flags == 1
    off = gb.with_geo_ref(False)
    assert not off.geo_ref and off.c_graph.flags == 0 and gb.c_graph.flags == 1
    bad = [dict(it) for it in items]
    bad[1]["edge_f"] = bad[1]["edge_f"].clone()
    bad[1]["edge_f"][5, 21] = 0.25  # one edge with a non-zero direction column
    gb2 = GraphBatch.from_arrays(bad, "cpu")
    assert not gb2.geo_ref and gb2.c_graph.flags == 0
    with pytest.raises(ValueError):
        gb2.with_geo_ref(True)
    assert not edge_feats_geo_ref(torch.zeros(4, 28)) and not edge_feats_geo_ref(None)


def test_geo_ref_claim_is_verified():
    """A caller's geo_ref=True is checked against the columns: wrong edge features raise instead of
    letting the kernels skip a branch that is not zero; the package-internal trusted
    path (device builder, select_graphs, concat_batches) carries the flag without a check."""
    from deepinteract_amd.graph import concat_batches, select_graphs
    z = load_case("tiny")
    items = [chain_item(z, "g1"), chain_item(z, "g2")]
    ok = GraphBatch.from_arrays(items, "cpu")
    args = (ok.src, ok.dst, ok.nbr, ok.node_f, ok.edge_f, ok.nodes_per_graph, ok.edges_per_graph)
    assert GraphBatch(*args, geo_ref=True).geo_ref
    assert not GraphBatch(*args, geo_ref=False).geo_ref
    ef = ok.edge_f.clone()
    ef[7, 21] = 0.5  # a non-zero direction column
    bad = (ok.src, ok.dst, ok.nbr, ok.node_f, ef, ok.nodes_per_graph, ok.edges_per_graph)
    with pytest.raises(ValueError):
        GraphBatch(*bad, geo_ref=True)
    assert not GraphBatch(*bad).geo_ref
    assert select_graphs(ok, [1, 0]).geo_ref and concat_batches([ok, ok]).geo_ref
    assert not select_graphs(ok.with_geo_ref(False), [0]).geo_ref


@pytest.mark.parametrize("case", ["tiny", "c1"])
def test_conformation_neighbour_messages_vanish(case):
    """The message branch of ConformationModule (oracle restatement of :384-418) is exactly zero
    for the reference featuriser's edges: dir_linear_1(dir_linear_0(0)) = 0, both bias-free."""
    z = load_case(case)
    sd = seeded_state_dict(0)
    it = chain_item(z, "g1")
    p = "gnn_module.0.gt_block.0.conformation_module"
    F_cur = torch.as_tensor(z["g1_init_edge"]) if "g1_init_edge" in z else torch.randn(it["edge_f"].shape[0], 128)
    src_ids, dst_ids = it["src_nbr"].permute(1, 0), it["dst_nbr"].permute(1, 0)
    nbr = torch.cat((F_cur[src_ids], F_cur[dst_ids]))
    nbr = F.silu(O._lin(nbr, sd, f"{p}.nbr_linear"))
    dist, dirf, ori, am = O._geo(it["edge_f"])
    am = am.reshape(-1, 1)
    nbr = nbr * O._lin(O._lin(dist, sd, f"{p}.dist_linear_0"), sd, f"{p}.dist_linear_1")
    nbr = F.silu(O._lin(nbr, sd, f"{p}.downward_proj"))
    gate = O._lin(O._lin(dirf, sd, f"{p}.dir_linear_0"), sd, f"{p}.dir_linear_1")
    assert torch.count_nonzero(gate) == 0
    msg = F.silu(O._lin(torch.sum(nbr * gate, dim=0), sd, f"{p}.upward_proj"))
    assert torch.count_nonzero(msg) == 0
    # and the module output is the one computed without the branch, bit for bit
    full = O.conformation(sd, p, it, F_cur, it["edge_f"])
    x = O._lin(F_cur, sd, f"{p}.orig_msg_linear")
    for b in range(2):
        x = O._resblock(sd, f"{p}.pre_res_blocks.{b}", x)
    x = F_cur + F.silu(O._lin(x, sd, f"{p}.res_connect_linear"))
    for b in range(2):
        x = O._resblock(sd, f"{p}.post_res_blocks.{b}", x)
    gsum = (O._lin(dist, sd, f"{p}.final_dist_linear") * x + O._lin(dirf, sd, f"{p}.final_dir_linear") * x
            + O._lin(ori, sd, f"{p}.final_orient_linear") * x + O._lin(am, sd, f"{p}.final_amide_linear") * x)
    assert torch.equal(full, F_cur + F.silu(O._lin(gsum, sd, f"{p}.final_linear")))


def test_init_edge_orientation_constants():
    """packing.init_blob's IEV_ORC / IEV_OGATE (fp32 blob: unscaled) equal InitEdge's orientation
    terms for orientation (0,0,0,1), and its direction terms are exactly zero."""
    sd = seeded_state_dict(0)
    p = "gnn_module.0.init_edge_module"
    _, vec, _, _ = init_blob(sd, "f32")
    ori = torch.tensor([[0.0, 0.0, 0.0, 1.0]], dtype=torch.float64)
    sd64 = {k: v.double() for k, v in sd.items()}
    t = GEO_ORDER.index("orient")
    wc0 = sd64[f"{p}.combined_linear_0.weight"]
    term0 = F.silu(ori @ sd64[f"{p}.orient_linear_0.weight"].T) @ wc0[:, 256 + 128 * t: 384 + 128 * t].T
    term1 = F.silu(ori @ sd64[f"{p}.orient_linear_1.weight"].T)
    np.testing.assert_allclose(vec[128:256].numpy(), term0[0].numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(vec[256:384].numpy(), term1[0].numpy(), rtol=1e-6, atol=1e-6)
    dirf = torch.zeros(1, 3, dtype=torch.float64)
    assert torch.count_nonzero(F.silu(dirf @ sd64[f"{p}.dir_linear_0.weight"].T)) == 0
    assert torch.count_nonzero(F.silu(dirf @ sd64[f"{p}.dir_linear_1.weight"].T)) == 0


def test_geo_ref_claim_on_a_batch_without_edges():
    """geo_ref=True on a batch with no edges takes the flag as False (nothing to skip), as the
    package-internal trusted path does, instead of raising."""
    import torch
    from deepinteract_amd.graph import GraphBatch
    n = 4
    empty = torch.zeros(0, dtype=torch.int32)
    gb = GraphBatch(empty, empty, torch.zeros(0, 4, dtype=torch.int32), torch.zeros(n, 113), torch.zeros(0, 28),
                    [n], [0], geo_ref=True)
    assert gb.geo_ref is False and gb.c_graph.flags == 0
    trusted = GraphBatch(empty, empty, torch.zeros(0, 4, dtype=torch.int32), torch.zeros(n, 113), torch.zeros(0, 28),
                         [n], [0], _trusted_geo_ref=True)
    assert trusted.geo_ref == gb.geo_ref
