"""The bf16 edge-layer kernel (k_edge_x32_ring: each wave's 32 edges as one v_mfma_f32_32x32x16_bf16
tile chain, weight stages on a 4-slot LDS ring shared by the 8 waves of a persistent block) against the golden vectors of the reference (tiny/c1/c2), and against the fp32 path
(k_edge_layer, exact-f32 MFMA; pinned to the oracle at C3 by test_gpu_c3.py) over EVERY node and
edge of a full C3 micro-batch (8 concatenated 2x1000 complexes).

Bounds: the stated bf16 bound (BF16_TOL, as test_gpu_parity.py) for both comparisons.
"""
import pytest
import torch

from gpu_common import chain_item, load_case, rel_max

pytestmark = pytest.mark.gpu

BF16_TOL = 1.5e-2


@pytest.fixture(scope="module")
def engines():
    from deepinteract_amd.engine import GeoTEngine
    from deepinteract_amd.weights import seeded_state_dict
    sd = seeded_state_dict(0)
    return {"bf16": GeoTEngine(sd, "bf16"), "f32": GeoTEngine(sd, "f32")}


@pytest.mark.parametrize("case", ["tiny", "c1", "c2"])
def test_edge_x32_matches_reference(engines, case):
    from deepinteract_amd.graph import GraphBatch
    z = load_case(case)
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    h, e = engines["bf16"].forward(gb)
    h, e = h.float().cpu().numpy(), e.float().cpu().numpy()
    n1, e1 = gb.nodes_per_graph[0], gb.edges_per_graph[0]
    errs = [rel_max(h[:n1], z["g1_node_out"]), rel_max(h[n1:], z["g2_node_out"]),
            rel_max(e[:e1][z["g1_edge_rows"]], z["g1_edge_out"]), rel_max(e[e1:][z["g2_edge_rows"]], z["g2_edge_out"])]
    print(f"{case} x32 bf16 GeoT node/edge errors:", ", ".join(f"{x:.3e}" for x in errs))
    assert max(errs) < BF16_TOL


@pytest.mark.parametrize("geo_ref", [True, False])
def test_edge_x32_vs_fp32_c3_microbatch(engines, geo_ref):
    """geo_ref False: the general path (neighbour gathers live, Fn rows written and read) on the
    same reference-featurised batch."""
    from deepinteract_amd import synth
    from deepinteract_amd.builder import build_graph_batch
    chains = [c for j in range(8) for c in synth.synthetic_complex(900 + j, 1000, 1000)]
    gb = build_graph_batch(chains, k=20, nbr_seeds=list(range(1, 17))).with_geo_ref(geo_ref)
    h0, e0 = engines["f32"].forward(gb)
    h1, e1 = engines["bf16"].forward(gb)
    torch.cuda.synchronize()
    assert torch.isfinite(h1.float()).all() and torch.isfinite(e1.float()).all()
    dn = rel_max(h1.float().cpu().numpy(), h0.cpu().numpy())
    de = rel_max(e1.float().cpu().numpy(), e0.cpu().numpy())
    print(f"C3 micro-batch x32 bf16 vs fp32 (geo_ref={geo_ref}): node {dn:.3e} edge {de:.3e}")
    assert dn < BF16_TOL and de < BF16_TOL
