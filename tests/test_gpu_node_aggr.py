"""Node-layer split (di_node_aggregate + di_node_update) vs the fused di_node_layer (bf16, round 6:
k_node_ws -- persistent weight-stationary blocks over 32-destination tiles; fp32: k_node_layer), and the CSR segment reduction itself vs an fp64 torch
reference on ragged in-degrees.

* split vs fused: bit-identical (same products, same edge order, same division, the same k-steps
  of every linear), fp32 and bf16, on the golden cases and on a full C3 micro-batch (8 x 2x1000
  residues, k = 20);
* di_node_aggregate vs fp64 torch on a ragged CSR (in-degrees 0..40, i.e. empty segments and
  segments spanning several 16-edge chunks): <= 1e-5 relative for fp32 V, and for bf16 V (the
  bf16 values are exact in fp32; only the fp32 accumulation rounds).
"""
import ctypes

import pytest
import torch

from gpu_common import chain_item, load_case

pytestmark = pytest.mark.gpu


def _engine(dtype):
    from deepinteract_amd.engine import GeoTEngine
    from deepinteract_amd.weights import seeded_state_dict
    return GeoTEngine(seeded_state_dict(0), dtype)


def _both(eng, gb):
    outs = []
    for split in (False, True):
        eng.split_node = split
        h, e = eng.forward(gb)
        torch.cuda.synchronize()
        outs.append((h, e))
    eng.split_node = True
    return outs


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("case", ["tiny", "c2"])
def test_split_node_layer_bit_identical(dtype, case):
    from deepinteract_amd.graph import GraphBatch
    z = load_case(case)
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    (h0, e0), (h1, e1) = _both(_engine(dtype), gb)
    assert torch.equal(h0, h1) and torch.equal(e0, e1)


def test_split_node_layer_bit_identical_c3_microbatch():
    from deepinteract_amd import synth
    from deepinteract_amd.builder import build_graph_batch
    chains = [c for j in range(8) for c in synth.synthetic_complex(950 + j, 1000, 1000)]
    gb = build_graph_batch(chains, k=20, nbr_seeds=list(range(1, 17)))
    (h0, e0), (h1, e1) = _both(_engine("bf16"), gb)
    assert torch.equal(h0, h1) and torch.equal(e0, e1)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_aggregate_ragged_csr(dtype):
    from deepinteract_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(7)
    n = 300
    deg = torch.randint(0, 41, (n,), generator=g)
    deg[:5] = torch.tensor([0, 1, 16, 17, 40])
    in_ptr = torch.zeros(n + 1, dtype=torch.int32)
    in_ptr[1:] = torch.cumsum(deg, 0)
    E = int(in_ptr[-1])
    src = torch.randint(0, n, (E,), generator=g, dtype=torch.int32)
    alpha = torch.exp(torch.empty(E, 4).uniform_(-5, 5, generator=g))
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    qkv = torch.randn(n, 384, generator=g).to(tdt)
    dev = torch.device("cuda")
    d_src, d_ptr, d_alpha, d_qkv = src.to(dev), in_ptr.to(dev), alpha.to(dev), qkv.to(dev)
    out = torch.full((n, 128), float("nan"), device=dev)
    cg = _lib.DiGraph(n, E, d_src.data_ptr(), None, None, None, d_ptr.data_ptr())
    rc = lib.di_node_aggregate(ctypes.byref(cg), _lib.DI_F32 if dtype == "f32" else _lib.DI_BF16,
                               d_alpha.data_ptr(), d_qkv.data_ptr(), out.data_ptr(),
                               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    # fp64 reference: wV / (z + 1e-6) per destination, heads of 32 features
    v = qkv[:, 256:].double()
    a = alpha.double().repeat_interleave(32, dim=1)               # [E, 128]
    dst = torch.repeat_interleave(torch.arange(n), deg)
    wv = torch.zeros(n, 128, dtype=torch.float64).index_add_(0, dst, a * v[src.long()])
    zz = torch.zeros(n, 128, dtype=torch.float64).index_add_(0, dst, a)
    ref = wv / (zz + 1e-6)
    got = out.double().cpu()
    assert torch.isfinite(got).all()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print(f"di_node_aggregate {dtype} ragged: {err:.3e}")
    assert err < 1e-5
    assert (got[deg == 0] == 0).all()


@pytest.mark.parametrize("final", [False, True])
def test_node_layer_ragged_csr_matches_split(final):
    """The bf16 di_node_layer (k_node_ws: persistent weight-stationary blocks, 32-destination tiles)
    on a ragged CSR -- in-degrees 0..40 (empty destinations, segments over several 8-edge chunks), a
    node count that leaves the last tile partial and more tiles than blocks -- bit-identical to the
    split form (di_node_aggregate + di_node_update) in h, Q|K|V and hT."""
    from deepinteract_amd import _lib
    lib = _lib.load()
    eng = _engine("bf16")
    nm, nv = eng.packed.node[1 if final else 0]
    g = torch.Generator().manual_seed(11)
    n = 32 * 300 + 13
    deg = torch.randint(0, 41, (n,), generator=g)
    deg[:6] = torch.tensor([0, 1, 8, 9, 17, 40])
    in_ptr = torch.zeros(n + 1, dtype=torch.int32)
    in_ptr[1:] = torch.cumsum(deg, 0)
    E = int(in_ptr[-1])
    src = torch.randint(0, n, (E,), generator=g, dtype=torch.int32)
    alpha = torch.exp(torch.empty(E, 4).uniform_(-5, 5, generator=g))
    dev = torch.device("cuda")
    qkv = torch.randn(n, 384, generator=g).to(torch.bfloat16).to(dev)
    h_in = torch.randn(n, 128, generator=g).to(torch.bfloat16).to(dev)
    d_src, d_ptr, d_alpha = src.to(dev), in_ptr.to(dev), alpha.to(dev)
    cg = _lib.DiGraph(n, E, d_src.data_ptr(), None, None, None, d_ptr.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for split in (False, True):
        h_out = torch.full((n, 128), float("nan"), dtype=torch.bfloat16, device=dev)
        q_out = None if final else torch.full((n, 384), float("nan"), dtype=torch.bfloat16, device=dev)
        hT = torch.full((128, n), float("nan"), dtype=torch.bfloat16, device=dev) if final else None
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        if split:
            attn = torch.empty(n, 128, device=dev)
            assert lib.di_node_aggregate(ctypes.byref(cg), _lib.DI_BF16, p(d_alpha), p(qkv), p(attn), st) == 0
            assert lib.di_node_update(ctypes.byref(cg), _lib.DI_BF16, int(final), p(attn), p(h_in), p(nm), p(nv),
                                      p(h_out), p(q_out), p(hT), st) == 0
        else:
            assert lib.di_node_layer(ctypes.byref(cg), _lib.DI_BF16, int(final), p(d_alpha), p(h_in), p(qkv), p(nm),
                                     p(nv), p(h_out), p(q_out), p(hT), st) == 0
        torch.cuda.synchronize()
        outs.append((h_out, q_out, hT))
    (h0, q0, t0), (h1, q1, t1) = outs
    assert torch.isfinite(h0.float()).all()
    assert torch.equal(h0, h1)
    if final:
        assert torch.equal(t0, t1) and torch.equal(t0, h0.t())
    else:
        assert torch.equal(q0, q1)
