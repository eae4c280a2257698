"""The grouped/lean bf16 edge-layer kernel (k_edge_lean, di_edge_config(1)) against the golden
vectors of the reference (tiny/c1/c2) and against the default kernel (k_edge_layer) on a full C3
micro-batch. Both kernels compute the same stage sequence with the same packed weights; they differ
in register residency, summation order inside fp32 accumulations (the edge FFN accumulates into its
residual, O_e adds the bias before the products) and hence in bf16 rounding only.

Bounds: vs the fp32 reference the stated bf16 bound (BF16_TOL, as test_gpu_parity.py); kernel 1 vs
kernel 0 (both bf16) the same bound over EVERY node and edge of 8 concatenated 2x1000 complexes.
"""
import pytest
import torch

from gpu_common import chain_item, load_case, rel_max

pytestmark = pytest.mark.gpu

BF16_TOL = 1.5e-2


@pytest.fixture(scope="module")
def eng():
    from deepinteract_amd.engine import GeoTEngine
    from deepinteract_amd.weights import seeded_state_dict
    return GeoTEngine(seeded_state_dict(0), "bf16")


def _with_kernel(k, fn):
    from deepinteract_amd import _lib
    lib = _lib.load()
    prev = lib.di_edge_config(k)
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        lib.di_edge_config(prev)


def test_edge_config_abi():
    from deepinteract_amd import _lib
    lib = _lib.load()
    cur = lib.di_edge_config(-1)
    assert cur in (0, 1)
    assert lib.di_edge_config(2) < 0 and lib.di_edge_config(-2) < 0
    assert lib.di_edge_config(-1) == cur


@pytest.mark.parametrize("case", ["tiny", "c1", "c2"])
def test_lean_matches_reference(eng, case):
    from deepinteract_amd.graph import GraphBatch
    z = load_case(case)
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    h, e = _with_kernel(1, lambda: eng.forward(gb))
    h, e = h.float().cpu().numpy(), e.float().cpu().numpy()
    n1, e1 = gb.nodes_per_graph[0], gb.edges_per_graph[0]
    errs = [rel_max(h[:n1], z["g1_node_out"]), rel_max(h[n1:], z["g2_node_out"]),
            rel_max(e[:e1][z["g1_edge_rows"]], z["g1_edge_out"]), rel_max(e[e1:][z["g2_edge_rows"]], z["g2_edge_out"])]
    print(f"{case} lean bf16 GeoT node/edge errors:", ", ".join(f"{x:.3e}" for x in errs))
    assert max(errs) < BF16_TOL


def test_lean_vs_default_c3_microbatch(eng):
    from deepinteract_amd import synth
    from deepinteract_amd.builder import build_graph_batch
    chains = [c for j in range(8) for c in synth.synthetic_complex(900 + j, 1000, 1000)]
    gb = build_graph_batch(chains, k=20, nbr_seeds=list(range(1, 17)))
    h0, e0 = _with_kernel(0, lambda: eng.forward(gb))
    h1, e1 = _with_kernel(1, lambda: eng.forward(gb))
    assert torch.isfinite(h1.float()).all() and torch.isfinite(e1.float()).all()
    dn = rel_max(h1.float().cpu().numpy(), h0.float().cpu().numpy())
    de = rel_max(e1.float().cpu().numpy(), e0.float().cpu().numpy())
    print(f"C3 micro-batch lean vs default (bf16 both): node {dn:.3e} edge {de:.3e}")
    assert dn < BF16_TOL and de < BF16_TOL
