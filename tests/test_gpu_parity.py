"""GPU parity of the HIP path against golden vectors produced by the reference's own code
(tests/golden/make_golden.py) and against the CPU oracle.

Tolerances (BASELINE.json north_star): fp32 outputs <= 1e-4 relative (max-abs error over the
tensor / max-abs of the reference tensor); kNN indices bit-exact. bf16 (stated looser bound):
GeoT node/edge outputs <= 1.5e-2 relative (measured <= 6.6e-3 on tiny/c1/c2), against
the same fp32 reference.
"""
import numpy as np
import pytest
import torch

from gpu_common import chain_arrays, chain_item, close_elem, load_case, logit_floor, rel_elem, rel_max

pytestmark = pytest.mark.gpu

CASES = ["tiny", "c1", "c2"]
F32_TOL = 1e-4
BF16_TOL = 1.5e-2  # measured <= 6.6e-3 (tiny/c1/c2); ~2x


@pytest.fixture(scope="module")
def sd():
    from deepinteract_amd.weights import seeded_state_dict
    return seeded_state_dict(0)


@pytest.fixture(scope="module")
def engines(sd):
    from deepinteract_amd.engine import GeoTEngine
    return {dt: GeoTEngine(sd, dt) for dt in ("f32", "bf16")}


def _batch(z):
    from deepinteract_amd.graph import GraphBatch
    return GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("geo_ref", [True, False])
def test_geot_matches_reference(engines, case, dtype, geo_ref):
    """geo_ref: the reference featuriser's constant direction / orientation columns are used
    (DI_GRAPH_GEO_REF: InitEdge's direction terms and the conformation messages skipped as exact
    zeros, orientation terms as constants) or the batch is forced onto the general path."""
    z = load_case(case)
    gb = _batch(z)
    assert gb.geo_ref
    if not geo_ref:
        gb = gb.with_geo_ref(False)
    h, e = engines[dtype].forward(gb)
    torch.cuda.synchronize()
    h, e = h.float().cpu().numpy(), e.float().cpu().numpy()
    n1 = gb.nodes_per_graph[0]
    e1 = gb.edges_per_graph[0]
    tol = F32_TOL if dtype == "f32" else BF16_TOL
    errs = [rel_max(h[:n1], z["g1_node_out"]), rel_max(h[n1:], z["g2_node_out"]),
            rel_max(e[:e1][z["g1_edge_rows"]], z["g1_edge_out"]), rel_max(e[e1:][z["g2_edge_rows"]], z["g2_edge_out"])]
    print(f"{case} {dtype} geo_ref={geo_ref} GeoT node/edge errors:", ", ".join(f"{x:.3e}" for x in errs))
    assert max(errs) < tol
    if dtype == "f32":
        np.testing.assert_allclose(e[:e1].astype(np.float64).sum(0), z["g1_edge_out_colsum"],
                                   rtol=1e-3, atol=1e-2 * np.abs(z["g1_edge_out_colsum"]).max())


@pytest.mark.parametrize("case", ["c1", "c2"])
def test_pair_tensor_exact(engines, case):
    from deepinteract_amd.engine import PairTensorOp
    z = load_case(case)
    gb = _batch(z)
    h, _ = engines["f32"].forward(gb)
    n1, n2 = gb.nodes_per_graph
    op = PairTensorOp()
    _, views = op(h, [0], [n1], [n1], [n2], hT=engines["f32"].last_hT)
    assert torch.equal(engines["f32"].last_hT, h.t())
    torch.cuda.synchronize()
    t = views[0]
    ref = torch.cat((h[:n1].t().unsqueeze(0).unsqueeze(3).expand(1, 128, n1, n2),
                     h[n1:].t().unsqueeze(0).unsqueeze(2).expand(1, 128, n1, n2)), 1)
    assert torch.equal(t, ref)
    # against the reference's pair tensor checksum / samples (fp32 tolerance)
    idx = torch.as_tensor(z["pair_sample_idx"]).long().cuda()
    samp = t[0, idx[:, 0], idx[:, 1], idx[:, 2]].cpu().numpy()
    assert rel_max(samp, z["pair_sample"]) < F32_TOL


def test_pair_tensor_batched_bf16_unaligned():
    """Ragged batch: 3 complexes of different (odd) sizes, bf16 -> scalar store path."""
    from deepinteract_amd.engine import PairTensorOp
    torch.manual_seed(0)
    sizes = [(7, 13), (20, 3), (33, 31)]
    rows = sum(a + b for a, b in sizes)
    h = torch.randn(rows, 128, device="cuda").to(torch.bfloat16)
    h1r, h2r, r = [], [], 0
    for a, b in sizes:
        h1r.append(r)
        h2r.append(r + a)
        r += a + b
    _, views = PairTensorOp()(h, h1r, h2r, [a for a, _ in sizes], [b for _, b in sizes])
    torch.cuda.synchronize()
    for (a, b), s1, s2, v in zip(sizes, h1r, h2r, views):
        ref = torch.cat((h[s1:s1 + a].t().unsqueeze(0).unsqueeze(3).expand(1, 128, a, b),
                         h[s2:s2 + b].t().unsqueeze(0).unsqueeze(2).expand(1, 128, a, b)), 1)
        assert torch.equal(v, ref)


def _pair_ref_check(h, sizes, h1r, h2r, views):
    for (a, b), s1, s2, v in zip(sizes, h1r, h2r, views):
        ref = torch.cat((h[s1:s1 + a].t().unsqueeze(0).unsqueeze(3).expand(1, 128, a, b),
                         h[s2:s2 + b].t().unsqueeze(0).unsqueeze(2).expand(1, 128, a, b)), 1)
        assert torch.equal(v, ref)


# every plane of these batches starts on a 128-B line (lines-eligible); row bytes 48 / 16 / 2000 /
# 8208 (bf16) and 16 / 4000 / 8208 (fp32) give periods of 8 rows = 3 / 1 / 125 / 513 lines
_LINES_SIZES = {torch.bfloat16: [(16, 24), (264, 8), (520, 1000), (8, 4104)],
                torch.float32: [(8, 4), (304, 1000), (8, 2052)]}
# 16-B aligned (row / vector kernels; the fp32 (12, 4) plane is not line aligned)
_ROW_SIZES = {torch.bfloat16: [(16, 24), (264, 8), (520, 1000), (8, 4104)],   # 4104: 5 row segments
              torch.float32: [(12, 4), (300, 1000), (4, 2052)]}


@pytest.mark.parametrize("kernel,waves,beside", [("lines", 4, False), ("lines", 2, True), ("lines", 1, False),
                                                 ("rows", 4, False), ("rows", 2, True), ("rows", 1, False),
                                                 ("vector", 4, False), ("auto", 0, False)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_pair_tensor_batched_aligned(dtype, kernel, waves, beside):
    """Ragged aligned batch through each aligned kernel and launch shape (every launch is the op's
    own: no process-wide state): planes spanning several row blocks / line periods, rows spanning
    several 128-chunk segments, varying L1/L2 per complex."""
    from deepinteract_amd.engine import PairTensorOp
    torch.manual_seed(1)
    sizes = (_LINES_SIZES if kernel in ("lines", "auto") else _ROW_SIZES)[dtype]
    rows = sum(a + b for a, b in sizes)
    h = torch.randn(rows, 128, device="cuda").to(dtype)
    h1r, h2r, r = [], [], 0
    for a, b in sizes:
        h1r.append(r)
        h2r.append(r + a)
        r += a + b
    op = PairTensorOp(kernel=kernel, waves_per_block=waves, beside=beside)
    _, views = op(h, h1r, h2r, [a for a, _ in sizes], [b for _, b in sizes], hT=h.t().contiguous())
    torch.cuda.synchronize()
    _pair_ref_check(h, sizes, h1r, h2r, views)


def test_pair_tensor_lines_refuses_unaligned_planes():
    """A 16-B-aligned batch whose planes do not start on 128-B lines: the lines kernel is refused
    (ValueError before any launch), auto takes the row kernel."""
    from deepinteract_amd.engine import PairTensorOp
    sizes = [(12, 4), (300, 1000)]
    h = torch.randn(sum(a + b for a, b in sizes), 128, device="cuda")
    h1r, h2r = [0, 16], [12, 316]
    with pytest.raises(ValueError):
        PairTensorOp(kernel="lines")(h, h1r, h2r, [12, 300], [4, 1000], hT=h.t().contiguous())
    _, views = PairTensorOp()(h, h1r, h2r, [12, 300], [4, 1000], hT=h.t().contiguous())
    torch.cuda.synchronize()
    _pair_ref_check(h, sizes, h1r, h2r, views)


@pytest.mark.parametrize("kernel,beside", [("lines", True), ("rows", False), ("vector", False)])
def test_pair_tensor_4096_square(kernel, beside):
    """The model limit (max_num_graph_nodes 4096): one 4096 x 4096 complex, bf16, [256, 4096, 4096]
    = 8.6 GB; plane = 2^24 elements (round 2 refused it with DI_ERANGE). Every channel plane is
    compared with its inputs, 32 channels at a time."""
    from deepinteract_amd.engine import PairTensorOp
    n = 4096
    torch.manual_seed(2)
    h = torch.randn(2 * n, 128, device="cuda").to(torch.bfloat16)
    out, views = PairTensorOp(kernel=kernel, beside=beside)(h, [0], [n], [n], [n], hT=h.t().contiguous())
    torch.cuda.synchronize()
    t = views[0][0]
    for c0 in range(0, 128, 32):
        assert torch.equal(t[c0:c0 + 32], h[:n, c0:c0 + 32].t().unsqueeze(2).expand(32, n, n))
        assert torch.equal(t[128 + c0:128 + c0 + 32], h[n:, c0:c0 + 32].t().unsqueeze(1).expand(32, n, n))
    del out, views, t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("case", ["knn1k", "tiny", "c1", "c2"])
def test_knn_bit_exact(case):
    from deepinteract_amd.builder import knn
    z = load_case(case)
    if case == "knn1k":
        chains = [(z["ca"], z["idx"], z["d2"])]
    else:
        chains = [(z[f"{t}_backbone"][:, 1, :], z[f"{t}_src"].reshape(-1, 20), z[f"{t}_d2"]) for t in ("g1", "g2")]
    cas = [torch.as_tensor(c[0]) for c in chains]
    idx, d2 = knn(cas, 20)
    torch.cuda.synchronize()
    off = 0
    for ca, ref_idx, ref_d2 in chains:
        n = ca.shape[0]
        got = idx[off:off + n].cpu().numpy()
        assert np.array_equal(got, ref_idx), f"{(got != ref_idx).sum()} mismatching neighbours"
        np.testing.assert_allclose(d2[off:off + n].cpu().numpy(), ref_d2, rtol=0, atol=2e-3)
        off += n


@pytest.mark.parametrize("case", ["tiny", "c1", "c2"])
def test_featuriser_matches_reference(case):
    from deepinteract_amd.builder import build_graph_batch
    z = load_case(case)
    chains = [chain_arrays(z, "g1"), chain_arrays(z, "g2")]
    gb, aux = build_graph_batch(chains, k=20, seed=1, device="cuda", return_aux=True)
    torch.cuda.synchronize()
    nf = gb.node_f.cpu().numpy()
    ef = gb.edge_f.cpu().numpy()
    n1 = gb.nodes_per_graph[0]
    e1 = gb.edges_per_graph[0]
    for tag, nsl, esl in (("g1", slice(0, n1), slice(0, e1)), ("g2", slice(n1, None), slice(e1, None))):
        rn, re_ = z[f"{tag}_node_f"], z[f"{tag}_edge_f"]
        np.testing.assert_allclose(nf[nsl], rn, rtol=0, atol=2e-4)
        got = ef[esl]
        np.testing.assert_allclose(got[:, :27], re_[:, :27], rtol=0, atol=2e-4)
        # amide-angle column: acos near +-1 amplifies 1-ulp differences of the normalised dot
        np.testing.assert_allclose(got[:, 27], re_[:, 27], rtol=0, atol=2e-3)
        src = gb.src.cpu().numpy()[esl] - (0 if tag == "g1" else n1)
        assert np.array_equal(src, z[f"{tag}_src"])


def test_nbr_ids_structure():
    from deepinteract_amd.builder import build_graph_batch
    z = load_case("c2")
    chains = [chain_arrays(z, "g1"), chain_arrays(z, "g2")]
    gb = build_graph_batch(chains, k=20, seed=7, device="cuda")
    nbr = gb.nbr.cpu().numpy().astype(np.int64)
    src = gb.src.cpu().numpy().astype(np.int64)
    dst = gb.dst.cpu().numpy().astype(np.int64)
    k = 20
    # global node v's in-edges are v*k .. v*k+k-1 (uniform in-degree)
    assert np.all(nbr[:, 0] // k == src) and np.all(nbr[:, 1] // k == src)
    assert np.all(nbr[:, 2] // k == dst) and np.all(nbr[:, 3] // k == dst)
    assert np.all(nbr[:, 0] != nbr[:, 1]) and np.all(nbr[:, 2] != nbr[:, 3])
    # roughly uniform over the k slots
    slots = np.bincount((nbr[:, 0] % k), minlength=k)
    assert slots.min() > 0.7 * slots.mean()
    gb2 = build_graph_batch(chains, k=20, seed=7, device="cuda")
    assert torch.equal(gb.nbr, gb2.nbr)  # deterministic for a seed


@pytest.mark.parametrize("case", ["tiny", "c1", "c2"])
def test_end_to_end_logits_f32(sd, case):
    """Built from the fixture's own graph tensors: GeoT (HIP) -> pair tensor (HIP) -> head (torch)."""
    from deepinteract_amd.modules import LitGINI
    z = load_case(case)
    model = LitGINI(dtype="f32", precise_head=True).cuda().eval()
    model.load_reference_state_dict(sd)
    from deepinteract_amd.graph import GraphBatch
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    with torch.no_grad():
        logits, probs = model.predict_batch(gb, [(0, 1)])
    torch.cuda.synchronize()
    assert rel_max(logits[0].cpu().numpy(), z["logits"]) < F32_TOL
    assert rel_max(probs[0].cpu().numpy(), z["probs"]) < F32_TOL
    # every contact probability within 1e-4 relative (north_star), elementwise; every logit within
    # 1e-4 relative + 1e-5 of max|logit| absolute (gpu_common.close_elem; logits cross zero, so the
    # floored relative figure is printed as the measured bound)
    lg = logits[0].cpu().numpy()
    pe = rel_elem(probs[0].cpu().numpy(), z["probs"])
    fl = logit_floor(z["logits"])
    le, lc = rel_elem(lg, z["logits"], fl), close_elem(lg, z["logits"])
    print(f"{case} fp32 contact probabilities: normwise {rel_max(probs[0].cpu().numpy(), z['probs']):.3e}, "
          f"elementwise relative {pe:.3e}; logits elementwise relative {le:.3e} (floor {fl:.3e}), "
          f"max abs {np.abs(lg - z['logits']).max():.3e}, allclose ratio {lc:.3f}")
    assert pe < F32_TOL
    assert lc <= 1.0


def test_geot_reference_init_weights():
    """Weights drawn the reference's way (glorot_orthogonal, zero biases, default BatchNorm;
    weights.reference_init_state_dict) through the HIP path vs the oracle, fp32."""
    import oracle.geot_oracle as O
    from deepinteract_amd.engine import GeoTEngine
    from deepinteract_amd.weights import reference_init_state_dict
    sd = reference_init_state_dict(1, with_head=False)
    z = load_case("tiny")
    gb = _batch(z)
    h, e = GeoTEngine(sd, "f32").forward(gb)
    torch.cuda.synchronize()
    h, e = h.cpu().numpy(), e.cpu().numpy()
    n1, e1 = gb.nodes_per_graph[0], gb.edges_per_graph[0]
    for tag, hs, es in (("g1", h[:n1], e[:e1]), ("g2", h[n1:], e[e1:])):
        it = chain_item(z, tag)
        g = {"num_nodes": it["num_nodes"], "src": it["src"], "dst": it["dst"], "src_nbr": it["src_nbr"],
             "dst_nbr": it["dst_nbr"], "node_f": it["node_f"].float(), "edge_f": it["edge_f"].float()}
        with torch.no_grad():
            hn, en = O.geot_forward(sd, g)
        assert rel_max(hs, hn.numpy()) < F32_TOL
        assert rel_max(es, en.numpy()) < F32_TOL


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_geot_general_path_nonzero_direction_features(engines, sd, dtype):
    """Edge features from a featuriser that is NOT the reference's (random direction /
    orientation columns): the batch is not DI_GRAPH_GEO_REF, the neighbour-message branch is live,
    and the whole GeoT still matches the oracle (fp32 <= 1e-4, bf16 within the stated bound)."""
    from deepinteract_amd.graph import GraphBatch
    from oracle import geot_oracle as O
    z = load_case("tiny")
    gen = torch.Generator().manual_seed(7)
    items = []
    for tag in ("g1", "g2"):
        it = chain_item(z, tag)
        ef = it["edge_f"].clone()
        ef[:, 20:23] = torch.randn(ef.shape[0], 3, generator=gen)
        ef[:, 23:27] = torch.nn.functional.normalize(torch.randn(ef.shape[0], 4, generator=gen), dim=-1)
        it["edge_f"] = ef
        items.append(it)
    gb = GraphBatch.from_arrays(items, "cuda")
    assert not gb.geo_ref and gb.c_graph.flags == 0
    h, e = engines[dtype].forward(gb)
    torch.cuda.synchronize()
    h, e = h.float().cpu().numpy(), e.float().cpu().numpy()
    tol = F32_TOL if dtype == "f32" else BF16_TOL
    errs = []
    for i, it in enumerate(items):
        with torch.no_grad():
            n_ref, e_ref = O.geot_forward(sd, it)
        n0, n1 = gb.node_off[i], gb.node_off[i + 1]
        e0, e1 = gb.edge_off[i], gb.edge_off[i + 1]
        errs += [rel_max(h[n0:n1], n_ref.numpy()), rel_max(e[e0:e1], e_ref.numpy())]
    print(f"tiny, random direction/orientation, {dtype}: node/edge errors", ", ".join(f"{x:.3e}" for x in errs))
    assert max(errs) < tol


def test_init_edge_resident_matches_staged(engines):
    """di_init_edge_resident (bf16 DI_GRAPH_GEO_REF batches without layer-0 Fn rows: the path's 128
    weight blocks resident in LDS, one block per CU, waves striding over 16-edge tiles with the next
    tile's indices prefetched) vs di_init_edge (staged weights). Same operands in the same order: F
    bit-identical. The batch (c2 concatenated 8x: 82k edges, 5120 tiles) gives several tiles per
    wave; a batch without the flag is refused."""
    import ctypes
    from deepinteract_amd import _lib
    from deepinteract_amd.engine import _ptr
    from deepinteract_amd.graph import concat_batches
    gb = concat_batches([_batch(load_case("c2"))] * 8)
    assert gb.geo_ref and gb.num_edges > 256 * 12 * 16
    eng = engines["bf16"]
    p, lib = eng.packed, eng.lib
    f_res = torch.full((gb.num_edges, 128), float("nan"), dtype=torch.bfloat16, device="cuda")
    f_stg = torch.full_like(f_res, float("nan"))
    _lib.check(lib.di_init_edge_resident(ctypes.byref(gb.c_graph), _ptr(gb.edge_f), _ptr(p.init[0]), _ptr(p.init[1]),
                                         _ptr(p.pos_src), _ptr(p.pos_dst), _ptr(f_res), None), "di_init_edge_resident")
    _lib.check(lib.di_init_edge(ctypes.byref(gb.c_graph), _lib.DI_BF16, _ptr(gb.edge_f), _ptr(p.init[0]),
                                _ptr(p.init[1]), _ptr(p.pos_src), _ptr(p.pos_dst), _ptr(f_stg), None, None),
               "di_init_edge")
    torch.cuda.synchronize()
    assert not torch.isnan(f_res.float()).any()
    assert torch.equal(f_res, f_stg)
    general = gb.with_geo_ref(False)
    assert lib.di_init_edge_resident(ctypes.byref(general.c_graph), _ptr(gb.edge_f), _ptr(p.init[0]), _ptr(p.init[1]),
                                     _ptr(p.pos_src), _ptr(p.pos_dst), _ptr(f_res), None) == -1


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_embed_init_edge_one_launch_matches_separate(engines, dtype):
    """di_embed_init_edge (the node embedding as the first blocks of the staged InitEdge launch) vs
    di_node_embed + di_init_edge: h, qkv and F bit-identical on the 8x-concatenated c2 batch, in
    both storage dtypes (fp32: the reference's precision, round 4)."""
    import ctypes
    from deepinteract_amd import _lib
    from deepinteract_amd.engine import _ptr
    from deepinteract_amd.graph import concat_batches
    gb = concat_batches([_batch(load_case("c2"))] * 8)
    eng = engines[dtype]
    p, lib = eng.packed, eng.lib
    di = _lib.DI_BF16 if dtype == "bf16" else _lib.DI_F32
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    g = ctypes.byref(gb.c_graph)
    n, e, d = gb.num_nodes, gb.num_edges, gb.node_f.shape[1]
    outs = []
    for fused in (True, False):
        h = torch.full((n, 128), float("nan"), dtype=tdt, device="cuda")
        qkv = torch.full((n, 384), float("nan"), dtype=tdt, device="cuda")
        f = torch.full((e, 128), float("nan"), dtype=tdt, device="cuda")
        if fused:
            _lib.check(lib.di_embed_init_edge(g, di, d, _ptr(gb.node_f), _ptr(p.embed[0]), _ptr(p.embed[1]), _ptr(h),
                                              _ptr(qkv), _ptr(gb.edge_f), _ptr(p.init[0]), _ptr(p.init[1]),
                                              _ptr(p.pos_src), _ptr(p.pos_dst), _ptr(f), None, -1, None),
                       "di_embed_init_edge")
        else:
            _lib.check(lib.di_node_embed(g, di, d, _ptr(gb.node_f), _ptr(p.embed[0]), _ptr(p.embed[1]),
                                         _ptr(h), _ptr(qkv), None, -1, None), "di_node_embed")
            _lib.check(lib.di_init_edge(g, di, _ptr(gb.edge_f), _ptr(p.init[0]), _ptr(p.init[1]),
                                        _ptr(p.pos_src), _ptr(p.pos_dst), _ptr(f), None, None), "di_init_edge")
        outs.append((h, qkv, f))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert not torch.isnan(a.float()).any()
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_pair_queue_ragged_jobs(dtype):
    """The pair queue (di_pair_signal / di_pair_stream / di_pair_help) over ragged jobs straight
    through the C ABI: complexes of different sizes in one job (empty 64-row blocks past a smaller
    chain 1, rows spanning several 128-chunk segments), jobs of different shapes, signals issued
    from the producer stream while the pair stream waits on the device, a help launch over the first
    jobs and the drain; every pair tensor bit-exact with its inputs."""
    import ctypes

    from deepinteract_amd import _lib
    from deepinteract_amd.pipeline import PairQueue
    lib = _lib.load()
    esz = torch.tensor([], dtype=dtype).element_size()
    vec = 16 // esz
    torch.manual_seed(3)
    job_sizes = [[(12, 8), (300, 1000)], [(65, 2064), (129, 24)], [(1, 8)], [(200, 200), (64, 64), (7, 1000)]]
    jobs, keep = [], []
    for sizes in job_sizes:
        rows = sum(-(-a // vec) * vec + b for a, b in sizes)
        h = torch.randn(rows, 128, device="cuda").to(dtype)
        hT = h.t().contiguous()
        h1r, h2r, r, off, descs = [], [], 0, 0, (_lib.DiPairDesc * len(sizes))()
        for i, (a, b) in enumerate(sizes):
            descs[i] = _lib.DiPairDesc(r, r + -(-a // vec) * vec, off, a, b)
            h1r.append(r)
            h2r.append(r + -(-a // vec) * vec)
            r += -(-a // vec) * vec + b
            off += 256 * a * b
        d = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).cuda()
        out = torch.full((off,), float("nan"), dtype=dtype, device="cuda")
        items = lib.di_pair_job_items(len(sizes), max(a for a, _ in sizes), 128)
        jobs.append(_lib.DiPairJob(hT.data_ptr(), d.data_ptr(), out.data_ptr(), rows, len(sizes),
                                   max(a for a, _ in sizes), items))
        keep.append((h, hT, d, out, sizes, h1r, h2r))
    q = PairQueue(torch.device("cuda"), len(jobs))
    q.set_jobs(jobs)
    di = _lib.DI_BF16 if dtype == torch.bfloat16 else _lib.DI_F32
    from deepinteract_amd.pipeline import schedule_streams
    main, side = schedule_streams()  # hardware queues of their own: the waiting stream never blocks main
    st = lambda s: ctypes.c_void_p(s.cuda_stream)  # noqa: E731
    qp, jp = ctypes.c_void_p(q.state.data_ptr()), ctypes.c_void_p(q.jobs.data_ptr())
    torch.cuda.synchronize()
    _lib.check(lib.di_pair_stream(di, jp, 0, len(jobs), 128, qp, None, 200.0, st(side)), "di_pair_stream")
    with torch.cuda.stream(main):
        for j in range(len(jobs)):
            torch.cuda._sleep(200000)  # the producer's work before each signal (~0.1 ms)
            _lib.check(lib.di_pair_signal(qp, j, st(main)), "di_pair_signal")
            if j == 1:
                _lib.check(lib.di_pair_help(di, jp, 0, 1, 128, qp, None, -1, st(main)), "di_pair_help")
        _lib.check(lib.di_pair_help(di, jp, 2, len(jobs) - 1, 128, qp, None, -1, st(main)), "di_pair_help (drain)")
    torch.cuda.synchronize()
    cnt = q.counters()
    total = sum(256 * a * b * esz for _, _, _, _, sizes, _, _ in keep for a, b in sizes)
    assert cnt["error"] == 0 and cnt["signalled"] == len(jobs) and cnt["stream_bytes"] + cnt["help_bytes"] == total, cnt
    assert cnt["gave_up"] == 0, cnt
    for h, _, _, out, sizes, h1r, h2r in keep:
        off = 0
        for (a, b), r1, r2 in zip(sizes, h1r, h2r):
            t = out[off:off + 256 * a * b].view(256, a, b)
            assert torch.equal(t[:128], h[r1:r1 + a].t().unsqueeze(2).expand(128, a, b))
            assert torch.equal(t[128:], h[r2:r2 + b].t().unsqueeze(1).expand(128, a, b))
            off += 256 * a * b
