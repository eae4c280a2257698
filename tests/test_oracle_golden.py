"""Pin the CPU oracle to the reference: golden vectors come from the reference's own modules
(tests/golden/make_golden.py). Expected: bit-exact (same fp32 op sequence on CPU)."""
import numpy as np
import pytest
import torch

from gpu_common import chain_arrays, chain_item, load_case, rel_max
from deepinteract_amd.weights import seeded_state_dict, state_dict_sha256
from oracle import geot_oracle as O


@pytest.fixture(scope="module")
def sd():
    return seeded_state_dict(0)


def test_weights_hash_matches_fixtures(sd):
    for case in ("tiny", "c1", "c2"):
        assert str(load_case(case)["weights_sha256"]) == state_dict_sha256(sd)


@pytest.mark.parametrize("case", ["tiny", "c1", "c2"])
def test_oracle_graph_builder_bit_exact(case):
    z = load_case(case)
    for tag in ("g1", "g2"):
        g = O.build_graph(chain_arrays(z, tag), seed=int(z[f"{tag}_nbr_seed"]))
        assert np.array_equal(g["src"].numpy(), z[f"{tag}_src"])
        assert np.array_equal(g["dst"].numpy(), z[f"{tag}_dst"])
        assert np.array_equal(g["src_nbr"].numpy(), z[f"{tag}_src_nbr"])
        assert np.array_equal(g["dst_nbr"].numpy(), z[f"{tag}_dst_nbr"])
        assert np.array_equal(g["node_f"].numpy(), z[f"{tag}_node_f"])
        assert np.array_equal(g["edge_f"].numpy(), z[f"{tag}_edge_f"])
        assert np.array_equal(g["d2"].numpy(), z[f"{tag}_d2"])


def test_oracle_knn_c3_size():
    z = load_case("knn1k")
    idx, d2 = O.knn(torch.as_tensor(z["ca"]))
    assert np.array_equal(idx.numpy(), z["idx"])
    assert np.array_equal(d2.numpy(), z["d2"])
    assert np.all(z["idx"][:, 0] == np.arange(z["idx"].shape[0]))  # self first


def test_known_answer_facts():
    z = load_case("c1")
    ef = z["g1_edge_f"]
    assert np.all(ef[:, 20:27] == np.array([0, 0, 0, 0, 0, 0, 1], dtype=np.float32))
    assert ef[:, 1].min() == 0.0 and ef[:, 1].max() == 1.0
    assert np.abs(z["g1_d2"][:, 0]).max() < 1e-2  # expansion-formula diagonal


@pytest.mark.parametrize("case", ["tiny", "c1", "c2"])
def test_oracle_geot_and_logits(sd, case):
    z = load_case(case)
    gs = []
    for tag in ("g1", "g2"):
        it = chain_item(z, tag)
        gs.append(dict(it, num_nodes=it["num_nodes"]))
    with torch.no_grad():
        logits, n1, e1, n2, e2 = O.predict(sd, gs[0], gs[1])
        probs = O.contact_probs(logits)
    assert rel_max(n1.numpy(), z["g1_node_out"]) < 1e-6
    assert rel_max(n2.numpy(), z["g2_node_out"]) < 1e-6
    assert rel_max(e1.numpy()[z["g1_edge_rows"]], z["g1_edge_out"]) < 1e-6
    assert rel_max(logits.numpy(), z["logits"]) < 1e-6
    assert rel_max(probs.numpy(), z["probs"]) < 1e-6


def test_oracle_intermediates_tiny(sd):
    z = load_case("tiny")
    it = chain_item(z, "g1")
    with torch.no_grad():
        n, e, inter = O.geot_forward(sd, it, return_intermediates=True)
    assert rel_max(inter["node_emb"].numpy(), z["g1_node_emb"]) < 1e-6
    assert rel_max(inter["init_edge"].numpy(), z["g1_init_edge"]) < 1e-6
    assert rel_max(inter["conf0"].numpy(), z["g1_conf0"]) < 1e-6
    assert rel_max(inter["node0"].numpy(), z["g1_layer0_node"]) < 1e-6
    assert rel_max(inter["edge0"].numpy(), z["g1_layer0_edge"]) < 1e-6
    assert rel_max(inter["conf1"].numpy(), z["g1_conf1"]) < 1e-6


def test_packed_blob_emulation_matches_reference(sd):
    """Host packing + BN folding + layout offsets, replayed densely on CPU (blob_emulator)."""
    from blob_emulator import Emu
    from deepinteract_amd.packing import PackedGeoT
    z = load_case("tiny")
    it = chain_item(z, "g1")
    h, e = Emu(PackedGeoT(sd, "f32")).geot(it)
    assert rel_max(h, z["g1_node_out"]) < 1e-5
    assert rel_max(e, z["g1_edge_out"]) < 1e-5


def test_packed_bf16_blob_emulation_log2_units(sd):
    """bf16 blobs carry the log2-unit SiLU scaling (packing.L2E; csrc/common.h silu2): replayed in
    float64 with the kernels' silu2 they reproduce the reference up to bf16 weight rounding."""
    from blob_emulator import Emu
    from deepinteract_amd.packing import PackedGeoT
    z = load_case("tiny")
    it = chain_item(z, "g1")
    h, e = Emu(PackedGeoT(sd, "bf16")).geot(it)
    assert rel_max(h, z["g1_node_out"]) < 2e-2
    assert rel_max(e, z["g1_edge_out"]) < 2e-2

