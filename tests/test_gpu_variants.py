"""The library's compile-time variants (tools/build_variants.py; built by __graft_entry__.build()
next to the product library) on the GPU, each in a child process that binds the variant instead of
the product build (deepinteract_amd._lib.load_variant):

* ``node2`` (DI_NODE_NW=2: k_node_layer in 2-wave blocks -- the round-2 fault's build): split vs
  fused node layer bit-identical in fp32 and bf16 on the c2 fixture, GeoT outputs vs the fixture;
* ``f32exact`` (DI_F32_FAST_SILU=0: fp32 SiLU as libm expf + IEEE division, the exact form the
  default build replaces with v_exp / v_rcp): fp32 GeoT node / edge outputs of tiny / c1 / c2 vs the
  reference's golden vectors within north_star's 1e-4.
"""
import os

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F32_TOL = 1e-4


def _variant(name):
    return os.path.join(ROOT, "deepinteract_amd", "lib", "variants", name, "libdeepinteract_amd.so")


def _geot_errors(eng, case):
    from gpu_common import chain_item, load_case, rel_max
    from deepinteract_amd.graph import GraphBatch
    z = load_case(case)
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    h, e = eng.forward(gb)
    h, e = h.float().cpu().numpy(), e.float().cpu().numpy()
    n1, e1 = gb.nodes_per_graph[0], gb.edges_per_graph[0]
    return [rel_max(h[:n1], z["g1_node_out"]), rel_max(h[n1:], z["g2_node_out"]),
            rel_max(e[:e1][z["g1_edge_rows"]], z["g1_edge_out"]), rel_max(e[e1:][z["g2_edge_rows"]], z["g2_edge_out"])]


def _child(name, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    try:
        import torch
        from deepinteract_amd import _lib
        _lib.load_variant(_variant(name))
        from deepinteract_amd.engine import GeoTEngine
        from deepinteract_amd.weights import seeded_state_dict
        sd = seeded_state_dict(0)
        out = {}
        if name == "node2":
            from gpu_common import chain_item, load_case
            from deepinteract_amd.graph import GraphBatch
            z = load_case("c2")
            gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
            for dt in ("f32", "bf16"):
                eng = GeoTEngine(sd, dt)
                res = []
                for split in (False, True):
                    eng.split_node = split
                    res.append(eng.forward(gb))
                torch.cuda.synchronize()
                out[f"{dt}_split_eq_fused"] = bool(torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1]))
                out[f"{dt}_errors"] = _geot_errors(eng, "c2")
        else:
            eng = GeoTEngine(sd, "f32")
            for case in ("tiny", "c1", "c2"):
                out[case] = _geot_errors(eng, case)
        q.put((out, None))
    except Exception as exc:
        q.put((None, repr(exc)))


def _run(name):
    path = _variant(name)
    assert os.path.exists(path), f"variant {name} not built: python tools/build_variants.py {name}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(name, q))
    p.start()
    try:
        out, err = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert err is None, err
    assert p.exitcode == 0
    print(name, out)
    return out


def test_variant_node2_two_wave_node_layer():
    out = _run("node2")
    assert out["f32_split_eq_fused"] and out["bf16_split_eq_fused"]
    assert max(out["f32_errors"]) < F32_TOL
    assert max(out["bf16_errors"]) < 1.5e-2


def test_variant_f32exact_matches_golden():
    out = _run("f32exact")
    for case in ("tiny", "c1", "c2"):
        assert max(out[case]) < F32_TOL, (case, out[case])
