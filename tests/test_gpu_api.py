"""The reference-shaped Python API on the GPU, against the golden vectors the
reference's own modules produced (tests/golden/make_golden.py):

* DGLGeometricTransformer.forward(graph)  deepinteract_modules.py:1426-1466 (in-place ndata/edata,
  batch_num_* kept)
* LitGINI.gnn_forward / shared_step(return_representations) / predict_step   :1660, :1687, :2178
* construct_interact_tensor  deepinteract_utils.py:158-172
* IndexError above max_num_graph_nodes (:153, :210), and a model with a larger positional table
* the per-stage intermediates of the tiny fixture through the module-at-a-time drop-ins
  (layers.py): InitEdgeModule, ConformationModule, GeometricTransformerModule
* load on the CPU, then .cuda() (lit_model_predict.py:214), and a CPU-resident model raising
* bf16 GeoT -> fp32 head end to end (stated bf16 logits / probability bounds)
* raw backbone arrays -> on-device builder with torch-seeded neighbour ids -> logits

fp32 tolerance 1e-4 relative (max-abs error / max-abs reference), as north_star states.
"""
import numpy as np
import pytest
import torch

from gpu_common import chain_arrays, chain_item, close_elem, load_case, logit_floor, rel_elem, rel_max

pytestmark = pytest.mark.gpu
F32_TOL = 1e-4
# bf16 GeoT (fp32 head) vs the fp32 reference, measured on MI355X: logits <= 1.32e-2
# relative (max-abs error / max-abs reference), contact probabilities <= 1.0e-2 absolute; bounds ~2x
BF16_LOGIT_TOL = 3e-2
BF16_PROB_ABS = 2e-2


@pytest.fixture(scope="module")
def sd():
    from deepinteract_amd.weights import seeded_state_dict
    return seeded_state_dict(0)


def residue_graph(z, tag, embed=None, device="cuda"):
    from deepinteract_amd.graph import ResidueGraph
    it = chain_item(z, tag)
    g = ResidueGraph(it["src"], it["dst"], it["num_nodes"])
    nf = it["node_f"]
    if embed is not None:
        nf = nf @ embed.t()
    g.ndata["f"] = nf
    g.edata["f"] = it["edge_f"]
    g.edata["src_nbr_e_ids"] = it["src_nbr"]
    g.edata["dst_nbr_e_ids"] = it["dst_nbr"]
    return g.to(device)


def _np(t):
    return t.detach().float().cpu().numpy()


@pytest.fixture(scope="module")
def model_f32(sd):
    from deepinteract_amd.modules import LitGINI
    return LitGINI(dtype="f32", precise_head=True).cuda().eval().load_reference_state_dict(sd)


@pytest.mark.parametrize("case", ["c1", "c2"])
def test_dgl_geometric_transformer_forward_in_place(sd, case):
    from deepinteract_amd.graph import batch
    from deepinteract_amd.modules import DGLGeometricTransformer
    z = load_case(case)
    emb = sd["node_in_embedding.weight"]
    g = batch([residue_graph(z, "g1", emb, "cpu"), residue_graph(z, "g2", emb, "cpu")]).to("cuda")
    bnn, bne = g.batch_num_nodes().clone(), g.batch_num_edges().clone()
    m = DGLGeometricTransformer(num_layers=2, dtype="f32").load_reference_state_dict(sd)
    out = m(g)
    torch.cuda.synchronize()
    assert out is g
    assert torch.equal(g.batch_num_nodes(), bnn) and torch.equal(g.batch_num_edges(), bne)
    n1, e1 = int(bnn[0]), int(bne[0])
    nf, ef = _np(g.ndata["f"]), _np(g.edata["f"])
    assert nf.shape == (n1 + int(bnn[1]), 128) and ef.shape == (e1 + int(bne[1]), 128)
    assert rel_max(nf[:n1], z["g1_node_out"]) < F32_TOL
    assert rel_max(nf[n1:], z["g2_node_out"]) < F32_TOL
    assert rel_max(ef[:e1][z["g1_edge_rows"]], z["g1_edge_out"]) < F32_TOL
    assert rel_max(ef[e1:][z["g2_edge_rows"]], z["g2_edge_out"]) < F32_TOL


@pytest.mark.parametrize("case", ["c1", "c2"])
def test_shared_step_and_predict_step(model_f32, case):
    z = load_case(case)
    g1, g2 = residue_graph(z, "g1"), residue_graph(z, "g2")
    with torch.no_grad():
        logits_list, g1_nf, g1_ef, g2_nf, g2_ef = model_f32.shared_step(g1, g2, return_representations=True)
    assert len(logits_list) == 1 and tuple(logits_list[0].shape) == tuple(z["logits"].shape)
    assert rel_max(_np(logits_list[0]), z["logits"]) < F32_TOL
    # every logit, elementwise: 1e-4 relative + 1e-5 of max|logit| absolute (gpu_common.close_elem)
    le = rel_elem(_np(logits_list[0]), z["logits"], logit_floor(z["logits"]))
    lc = close_elem(_np(logits_list[0]), z["logits"])
    print(f"{case} shared_step logits elementwise relative {le:.3e} (floored), allclose ratio {lc:.3f}")
    assert lc <= 1.0
    for nf, ef, tag in ((g1_nf, g1_ef, "g1"), (g2_nf, g2_ef, "g2")):
        assert isinstance(nf, np.ndarray) and isinstance(ef, np.ndarray)
        assert rel_max(nf, z[f"{tag}_node_out"]) < F32_TOL
        assert rel_max(ef[z[f"{tag}_edge_rows"]], z[f"{tag}_edge_out"]) < F32_TOL
    # the graphs were updated in place, as DGLGeometricTransformer.forward does
    assert rel_max(_np(g1.ndata["f"]), z["g1_node_out"]) < F32_TOL
    # predict_step(batch) = shared_step(graph1, graph2, return_representations=True)
    g1, g2 = residue_graph(z, "g1"), residue_graph(z, "g2")
    with torch.no_grad():
        out = model_f32.predict_step((g1, g2), 0)
    assert rel_max(_np(out[0][0]), z["logits"]) < F32_TOL
    from deepinteract_amd.head import contact_probs
    assert rel_max(_np(contact_probs(out[0][0])), z["probs"]) < F32_TOL
    # elementwise relative error of every contact probability (north_star: <= 1e-4 relative)
    pe = rel_elem(_np(contact_probs(out[0][0])), z["probs"])
    print(f"{case} predict_step contact probabilities: elementwise relative {pe:.3e}")
    assert pe < F32_TOL


def test_gnn_forward_batched_graphs(model_f32):
    """gnn_forward on a dgl.batch of two chains returns per-chain node features (dgl.unbatch)."""
    from deepinteract_amd.graph import batch
    z = load_case("c1")
    g = batch([residue_graph(z, "g1", device="cpu"), residue_graph(z, "g2", device="cpu")]).to("cuda")
    with torch.no_grad():
        feats = model_f32.gnn_forward(g)
    assert len(feats) == 2
    assert rel_max(_np(feats[0]), z["g1_node_out"]) < F32_TOL
    assert rel_max(_np(feats[1]), z["g2_node_out"]) < F32_TOL


@pytest.mark.parametrize("case", ["c1", "c2"])
def test_construct_interact_tensor(case):
    from deepinteract_amd.modules import construct_interact_tensor
    z = load_case(case)
    a = torch.as_tensor(z["g1_node_out"]).cuda()
    b = torch.as_tensor(z["g2_node_out"]).cuda()
    t = construct_interact_tensor(a, b)
    torch.cuda.synchronize()
    assert tuple(t.shape) == tuple(z["pair_shape"])
    idx = torch.as_tensor(z["pair_sample_idx"]).long().cuda()
    samp = _np(t[0, idx[:, 0], idx[:, 1], idx[:, 2]])
    assert np.array_equal(samp, z["pair_sample"])  # a copy of the same fp32 values
    assert abs(float(t.double().sum()) - float(z["pair_sum"])) <= 1e-6 * abs(float(z["pair_sum"])) + 1e-3


def test_index_error_above_node_count_limit(model_f32):
    from deepinteract_amd.graph import ResidueGraph
    n, k = 2305, 20
    dst = torch.arange(n).repeat_interleave(k)
    src = (dst + torch.arange(k).repeat(n)) % n
    g = ResidueGraph(src, dst, n, device="cuda")
    g.ndata["f"] = torch.zeros(n, 113, device="cuda")
    g.edata["f"] = torch.zeros(n * k, 28, device="cuda")
    g.edata["src_nbr_e_ids"] = torch.zeros(n * k, 2, dtype=torch.long, device="cuda")
    g.edata["dst_nbr_e_ids"] = torch.zeros(n * k, 2, dtype=torch.long, device="cuda")
    with pytest.raises(IndexError):
        model_f32.gnn_forward(g)


def test_larger_positional_table_through_litgini():
    """max_num_graph_nodes=4096 (C5 class): a 2400-residue chain passes through LitGINI.gnn_forward
    and gives exactly what GeoTEngine gives on the same device-built graph."""
    from deepinteract_amd import synth
    from deepinteract_amd.builder import build_graph_batch
    from deepinteract_amd.config import GeoTConfig
    from deepinteract_amd.engine import GeoTEngine
    from deepinteract_amd.graph import ResidueGraph
    from deepinteract_amd.modules import LitGINI
    from deepinteract_amd.weights import seeded_state_dict
    cfg = GeoTConfig(node_count_limit=4096)
    sd4 = seeded_state_dict(3, cfg)
    m = LitGINI(dtype="f32", max_num_graph_nodes=4096).cuda().eval().load_reference_state_dict(sd4)
    ch = synth.synthetic_chain(2400, 42)
    gb = build_graph_batch([ch], nbr_seeds=[5], node_count_limit=4096)
    g = ResidueGraph(gb.src.long(), gb.dst.long(), gb.num_nodes, device="cuda")
    g.ndata["f"], g.edata["f"] = gb.node_f, gb.edge_f
    g.edata["src_nbr_e_ids"], g.edata["dst_nbr_e_ids"] = gb.nbr[:, :2].long(), gb.nbr[:, 2:].long()
    with torch.no_grad():
        feats = m.gnn_forward(g)
        ref, _ = GeoTEngine(sd4, "f32", cfg).forward(gb)
    torch.cuda.synchronize()
    assert torch.equal(feats[0], ref)


@pytest.mark.parametrize("stage", ["init_edge", "conf0", "layer0", "conf1"])
def test_tiny_reference_intermediates(sd, stage):
    """Per-stage parity on the reference-made intermediates of the tiny fixture (module hooks in
    make_golden.py), through the module-at-a-time drop-ins at fp32."""
    from deepinteract_amd import layers
    z = load_case("tiny")
    sub = lambda pre: {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}  # noqa: E731
    for tag in ("g1", "g2"):
        g = residue_graph(z, tag)
        G = g.edata["f"]
        if stage == "init_edge":
            m = layers.InitEdgeModule("f32").load_reference_state_dict(sub("gnn_module.0.init_edge_module."))
            got, want = m(g), z[f"{tag}_init_edge"]
        elif stage == "conf0":
            g.edata["f"] = torch.as_tensor(z[f"{tag}_init_edge"]).cuda()
            m = layers.ConformationModule("f32").load_reference_state_dict(
                sub("gnn_module.0.gt_block.0.conformation_module."))
            got, want = m(g, G), z[f"{tag}_conf0"]
        elif stage == "layer0":
            g.ndata["f"] = torch.as_tensor(z[f"{tag}_node_emb"]).cuda()
            g.edata["f"] = torch.as_tensor(z[f"{tag}_init_edge"]).cuda()
            m = layers.GeometricTransformerModule("f32").load_reference_state_dict(sub("gnn_module.0.gt_block.0."))
            node, edge = m(g, G)
            assert rel_max(_np(edge), z[f"{tag}_layer0_edge"]) < F32_TOL
            got, want = node, z[f"{tag}_layer0_node"]
        else:
            g.edata["f"] = torch.as_tensor(z[f"{tag}_layer0_edge"]).cuda()
            m = layers.ConformationModule("f32").load_reference_state_dict(
                sub("gnn_module.0.gt_block.1.conformation_module."))
            got, want = m(g, G), z[f"{tag}_conf1"]
        assert rel_max(_np(got), want) < F32_TOL, (tag, stage)


def test_load_on_cpu_then_cuda(tmp_path, sd):
    """lit_model_predict.py:214 loads without map_location and moves the model afterwards."""
    import os
    from deepinteract_amd.graph import GraphBatch
    from deepinteract_amd.modules import LitGINI
    z = load_case("tiny")
    p = os.path.join(tmp_path, "LitGINI.ckpt")
    torch.save({"state_dict": sd, "hyper_parameters": {"num_gnn_layers": 2, "knn": 20}}, p)
    model = LitGINI.load_from_checkpoint(p, precise_head=True).freeze()
    assert next(model.parameters()).device.type == "cpu"
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    with pytest.raises(RuntimeError):
        model.predict_batch(gb, [(0, 1)])  # still on the CPU: refuses instead of passing host pointers
    model = model.cuda()
    with torch.no_grad():
        logits, probs = model.predict_batch(gb, [(0, 1)])
    torch.cuda.synchronize()
    assert rel_max(_np(logits[0]), z["logits"]) < F32_TOL
    assert rel_max(_np(probs[0]), z["probs"]) < F32_TOL


@pytest.mark.parametrize("case", ["c1", "c2"])
def test_bf16_geot_fp32_head_end_to_end(sd, case):
    from deepinteract_amd.graph import GraphBatch
    from deepinteract_amd.modules import LitGINI
    z = load_case(case)
    model = LitGINI(dtype="bf16", precise_head=True).cuda().eval().load_reference_state_dict(sd)
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    with torch.no_grad():
        logits, probs = model.predict_batch(gb, [(0, 1)])
    torch.cuda.synchronize()
    el = rel_max(_np(logits[0]), z["logits"])
    ep = float(np.abs(_np(probs[0]) - z["probs"]).max())
    print(f"{case} bf16 GeoT + fp32 head: logits rel {el:.3e}, probs abs {ep:.3e}")
    assert el < BF16_LOGIT_TOL and ep < BF16_PROB_ABS


@pytest.mark.parametrize("case", ["tiny", "c1", "c2"])
def test_raw_arrays_through_builder_to_logits(model_f32, case):
    """Backbone / amide / DIPS arrays -> on-device builder with the fixture's torch seeds ->
    neighbour ids bit-exact with the reference's -> GeoT -> head: logits within 1e-4."""
    from deepinteract_amd.builder import build_graph_batch
    z = load_case(case)
    seeds = [int(z["g1_nbr_seed"]), int(z["g2_nbr_seed"])]
    gb = build_graph_batch([chain_arrays(z, "g1"), chain_arrays(z, "g2")], nbr_seeds=seeds)
    nbr = gb.nbr.cpu().numpy()
    n1, e1 = gb.nodes_per_graph[0], gb.edges_per_graph[0]
    assert np.array_equal(nbr[:e1, :2], z["g1_src_nbr"]) and np.array_equal(nbr[:e1, 2:], z["g1_dst_nbr"])
    assert np.array_equal(nbr[e1:, :2] - e1, z["g2_src_nbr"]) and np.array_equal(nbr[e1:, 2:] - e1, z["g2_dst_nbr"])
    assert np.array_equal(gb.src.cpu().numpy()[:e1], z["g1_src"])
    with torch.no_grad():
        logits, probs = model_f32.predict_batch(gb, [(0, 1)])
    torch.cuda.synchronize()
    el = rel_max(_np(logits[0]), z["logits"])
    print(f"{case} raw arrays -> builder -> logits rel {el:.3e}")
    assert el < F32_TOL
    assert rel_max(_np(probs[0]), z["probs"]) < F32_TOL


@pytest.mark.parametrize("k,n", [(3, 97), (7, 300), (20, 1000)])
def test_torch_seeded_nbr_ids_vs_torch_randperm(k, n):
    """di_build_nbr_ids_torch against torch's own CPU generator: after torch.manual_seed(seed) the
    reference draws randperm(k) once per edge for the src side, then once per edge for the dst
    side, and keeps the first two entries as positions in the endpoint's in-edge list
    (deepinteract_utils.py:539-546; in-edges of v are v*k .. v*k+k-1). Two chains per batch, so
    the second chain's ids carry the batch edge offset."""
    from deepinteract_amd import synth
    from deepinteract_amd.builder import build_graph_batch
    chains = list(synth.synthetic_complex(11, n, n + 5))
    seeds = [1234, 99]
    gb = build_graph_batch(chains, k=k, nbr_seeds=seeds)
    nbr = gb.nbr.cpu().numpy()
    src, dst = gb.src.cpu().numpy(), gb.dst.cpu().numpy()
    for g, seed in enumerate(seeds):
        e0, e1 = gb.edge_off[g], gb.edge_off[g + 1]
        E = e1 - e0
        torch.manual_seed(seed)
        p_src = torch.stack([torch.randperm(k)[:2] for _ in range(E)]).numpy()
        p_dst = torch.stack([torch.randperm(k)[:2] for _ in range(E)]).numpy()
        want = np.concatenate([src[e0:e1, None] * k + p_src, dst[e0:e1, None] * k + p_dst], 1)
        assert np.array_equal(nbr[e0:e1], want), (k, n, g)
