"""Host-only calls into the C ABI, run in a child process against the ASan/UBSan build of the library
(tests/test_host_sanitizers.py). Every call below returns before any kernel launch: argument
validation (NULL pointers, bad dtypes / shapes / flags / launch structs), size queries and the
pair-tensor shape check, at the edges of every range the host code computes with (int32 products,
64-bit plane and work-space sizes). No torch import, no GPU.

usage: python host_abi_calls.py <library path>    (exit 0 and "host ABI calls: N ok" on success)
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deepinteract_amd import _lib  # noqa: E402  (ctypes binding only; no torch)

I32_MAX = 2**31 - 1
EINVAL, ERANGE = -1, -2


def main(path):
    lib = _lib._bind(path)
    n = 0

    def expect(got, want, what):
        nonlocal n
        if got != want:
            raise SystemExit(f"{what}: got {got}, want {want}")
        n += 1

    p = ctypes.c_void_p(16)  # never dereferenced on these paths
    expect(lib.di_abi_version(), _lib.ABI_VERSION, "abi")
    # size queries (int64 arithmetic)
    for kind in range(7):
        for dt in (_lib.DI_F32, _lib.DI_BF16):
            for vec in (0, 1):
                got = lib.di_blob_bytes(kind, dt, vec)
                if got <= 0:
                    raise SystemExit(f"blob bytes {kind} {dt} {vec}: {got}")
                n += 1
    expect(lib.di_blob_bytes(7, 0, 0), -1, "blob kind")
    expect(lib.di_blob_bytes(-1, 0, 0), -1, "blob kind")
    expect(lib.di_blob_bytes(0, 5, 0), -1, "blob dtype")
    expect(lib.di_head_prologue_work_bytes(8, 1000, 900, 128), 8 * 128 * (2 * 1900 * 4 + 4), "prologue work")
    expect(lib.di_head_prologue_work_bytes(65535, 65535, 65535, 65535) > 0, True, "prologue work, large")
    expect(lib.di_head_prologue_work_bytes(0, 10, 10, 128), 0, "prologue work, empty")
    expect(lib.di_inorm_work_bytes(128, 1 << 40) > 0, True, "inorm work, large")
    # pair tensor: shape / launch validation
    L = _lib.DiPairLaunch
    for args, want in (((1, 4096, 4096, 128, 2), 0), ((8, 4096, 4096, 128, 4), 0), ((1, 32768, 32768, 128, 2), ERANGE),
                       ((1, I32_MAX, I32_MAX, I32_MAX, 4), ERANGE), ((I32_MAX, 1000, 1000, 128, 2), ERANGE),
                       ((1, 1 << 21, 8, 128, 2), ERANGE), ((0, 10, 10, 128, 2), EINVAL), ((1, -5, 10, 128, 2), EINVAL),
                       ((1, 10, 10, 128, 3), EINVAL)):
        expect(lib.di_pair_tensor_check(*args, None), want, f"pair check {args}")
    for launch, want in ((L(3, 0, 2, 1), 0), (L(4, 0, 0, 0), EINVAL), (L(-1, 0, 0, 0), EINVAL),
                         (L(0, -1, 0, 0), EINVAL), (L(0, 0, 17, 0), EINVAL), (L(0, 0, 0, 2), EINVAL),
                         (L(0, I32_MAX, 16, 1), 0)):
        expect(lib.di_pair_tensor_check(1, 64, 64, 128, 2, ctypes.byref(launch)), want, "pair launch")
    for kernel, aligned in ((_lib.DI_PAIR_LINES, 1), (_lib.DI_PAIR_ROWS, 0), (_lib.DI_PAIR_VECTOR, 0)):
        launch = L(kernel, 0, 0, 0)
        expect(lib.di_pair_tensor(1, p, 1, 64, 64, 128, aligned, p, p, 128, ctypes.byref(launch), p, None), EINVAL,
               f"pair kernel {kernel} at aligned {aligned}")
    expect(lib.di_pair_tensor(1, p, 1, 64, 64, 128, 3, p, p, 128, None, p, None), EINVAL, "pair aligned flag")
    expect(lib.di_pair_tensor(1, p, 1, 64, 64, 128, 1, p, None, 128, None, p, None), EINVAL, "pair hT")
    expect(lib.di_pair_tensor(1, None, 1, 64, 64, 128, 1, p, p, 128, None, p, None), EINVAL, "pair descs")
    expect(lib.di_pair_tensor(7, p, 1, 64, 64, 128, 1, p, p, 128, None, p, None), EINVAL, "pair dtype")
    expect(lib.di_pair_tensor(1, p, 1, 1 << 21, 8, 128, 1, p, p, 128, None, p, None), ERANGE, "pair range")
    # GeoT entry points: NULL graph / pointers, empty graphs, bad dtype, Fn contract
    G = _lib.DiGraph
    for g in (G(8, 16, 16, 16, 16, 16, 16, 0), G(0, 0, 16, 16, 16, 16, 16, 0), G(-1, -20, 16, 16, 16, 16, 16, 1)):
        gp = ctypes.byref(g)
        expect(lib.di_node_embed(gp, 1, 0, p, p, p, p, p, None, -1, None), EINVAL, "embed in_dim")
        expect(lib.di_node_embed(gp, 1, 129, p, p, p, p, p, None, -1, None), EINVAL, "embed in_dim > 128")
        expect(lib.di_node_embed(gp, 9, 113, p, p, p, p, p, None, -1, None), EINVAL, "embed dtype")
        expect(lib.di_node_embed(gp, 1, 113, None, p, p, p, p, None, -1, None), EINVAL, "embed NULL")
        expect(lib.di_init_edge(gp, 1, p, p, p, p, p, p, None, None), EINVAL, "init Fn")
        expect(lib.di_init_edge(gp, 9, p, p, p, p, p, p, p, None), EINVAL, "init dtype")
        expect(lib.di_init_edge_resident(gp, p, p, p, p, p, None, None), EINVAL, "init resident f_out")
        expect(lib.di_embed_init_edge(gp, 1, 129, p, p, p, p, p, p, p, p, p, p, p, None, -1, None), EINVAL, "embed+init in_dim")
        expect(lib.di_embed_init_edge(gp, 6, 113, p, p, p, p, p, p, p, p, p, p, p, None, -1, None), EINVAL, "embed+init dtype")
        expect(lib.di_edge_layer(gp, 1, 0, p, p, None, p, p, p, p, p, p, None), EINVAL, "edge Fn in")
        expect(lib.di_edge_layer(gp, 1, 0, p, p, p, p, p, p, p, p, None, None), EINVAL, "edge Fn out")
        expect(lib.di_edge_layer(gp, 1, 0, p, p, p, p, p, p, p, None, p, None), EINVAL, "edge f_out")
        expect(lib.di_edge_layer(gp, 4, 1, p, p, p, p, p, p, p, None, None, None), EINVAL, "edge dtype")
        expect(lib.di_node_layer(gp, 1, 0, p, p, p, p, p, p, None, None, None), EINVAL, "node qkv_out")
        expect(lib.di_node_layer(gp, 3, 1, p, p, p, p, p, p, None, None, None), EINVAL, "node dtype")
        expect(lib.di_node_update(gp, 1, 0, p, p, p, p, p, None, None, None), EINVAL, "update qkv_out")
        expect(lib.di_edge_layer_attn(gp, 0, 1, p, p, p, p, p, p, None, None, None, p, p, None), EINVAL,
               "edge attn f32")
        expect(lib.di_edge_layer_attn(gp, 1, 1, p, p, p, p, p, p, None, None, None, None, p, None), EINVAL,
               "edge attn NULL attn")
        expect(lib.di_edge_layer_attn(gp, 1, 1, p, p, p, p, p, p, None, None, None, p, None, None), EINVAL,
               "edge attn NULL parts")
        expect(lib.di_edge_layer_attn(gp, 1, 0, p, p, p, p, p, p, None, None, None, p, p, None), EINVAL,
               "edge attn f_out")
        expect(lib.di_node_update_folded(gp, 1, 1, p, None, p, p, p, p, None, None, None), EINVAL,
               "update folded NULL parts")
        expect(lib.di_node_aggregate(gp, 1, None, p, p, None), EINVAL, "aggregate NULL")
        expect(lib.di_conformation(gp, 1, p, p, None, p, p, p, None), EINVAL, "conformation Fn")
        expect(lib.di_geo_attention(gp, 1, None, p, p, p, p, None), EINVAL, "attention NULL")
    # every graph entry point with a NULL graph (remaining arguments plausible)
    for fn in ("di_node_embed", "di_init_edge", "di_init_edge_resident", "di_embed_init_edge", "di_edge_layer", "di_node_layer", "di_node_aggregate",
               "di_node_update", "di_conformation", "di_geo_attention", "di_edge_layer_attn", "di_node_update_folded"):
        argtypes = _lib._SIGS[fn][0]
        args = [None] + [1 if t is _lib._I else p for t in argtypes[1:]]
        args[-1] = None  # stream
        expect(getattr(lib, fn)(*args), EINVAL, f"{fn} NULL graph")
    # fold partial-sum buffer: ceil(Et / 32) tiles x 2 slots x 132 floats
    expect(lib.di_attn_parts_bytes(0), EINVAL, "attn parts empty")
    expect(lib.di_attn_parts_bytes(33), 2 * 2 * 132 * 4, "attn parts 33 edges")
    expect(lib.di_attn_parts_bytes(32), 1 * 2 * 132 * 4, "attn parts 32 edges")
    # builder entry points: range checks in int32 / int64 arithmetic
    expect(lib.di_knn_topk(1, None, None, 20, 10, None, None, None), EINVAL, "knn NULL")
    expect(lib.di_knn_topk(1, p, p, 20, 4097, p, p, None), EINVAL, "knn max nodes")
    expect(lib.di_knn_topk(70000, p, p, 20, 100, p, p, None), EINVAL, "knn graphs")
    expect(lib.di_knn_graph(1, p, 20, p, I32_MAX, p, p, p, p, None), EINVAL, "knn graph int32 edges")
    expect(lib.di_build_nbr_ids_torch(1, p, 20, p, I32_MAX // 20, p, p, p, None), ERANGE, "nbr draws int32")
    expect(lib.di_build_nbr_ids_torch(1, p, 20, p, 2_900_000, p, p, p, None), ERANGE, "nbr draws int32 edge")
    expect(lib.di_build_nbr_ids_torch(1, p, 2, p, 100, p, p, p, None), EINVAL, "nbr k < 3")
    expect(lib.di_build_nbr_ids_torch(1, p, 257, p, 100, p, p, p, None), EINVAL, "nbr k > 256")
    expect(lib.di_build_nbr_ids(0, p, p, p, 1, p, None), EINVAL, "nbr counter empty")
    ga = _lib.DiGeoArgs(0, 20, 10, 16, 16, 16, 16, 16, 16, 16, 16, 16)
    expect(lib.di_geo_feats(ctypes.byref(ga), None), EINVAL, "geo feats empty")
    expect(lib.di_geo_feats(None, None), EINVAL, "geo feats NULL")
    # head ops
    expect(lib.di_head_prologue(0, None, 1, 8, 8, 128, 128, 1, None, None, None, None, None, 1e-6, None, None, None),
           EINVAL, "prologue NULL")
    expect(lib.di_head_prologue(1, p, 1, 8, 8, 130, 128, 1, p, p, p, p, p, 1e-6, p, p, None), EINVAL, "prologue hidden")
    expect(lib.di_head_prologue(1, p, 1, 65536, 65536, 128, 128, 1, p, p, p, p, p, 1e-6, p, p, None), ERANGE,
           "prologue range")
    expect(lib.di_inorm_elu(1, None, 128, 100, p, p, 1e-5, p, p, None), EINVAL, "inorm NULL")
    expect(lib.di_se_scale_add(1, None, p, p, p, 128, 100, p, None), EINVAL, "se NULL")
    expect(lib.di_channel_mean(1, None, 128, 100, p, p, p, None), EINVAL, "mean NULL")
    expect(lib.di_gemm_bias_act(1, 0, 128, 128, p, 128, p, p, 0, p, 128, p, 128, None), EINVAL, "gemm rows")
    expect(lib.di_gemm_bias_act(2, 64, 128, 128, p, 128, p, p, 0, p, 128, p, 128, None), EINVAL, "gemm dtype")
    expect(lib.di_inorm_elu(6, p, 128, 100, p, p, 1e-5, p, p, None), EINVAL, "inorm dtype")
    expect(lib.di_head_prologue(3, p, 1, 8, 8, 128, 128, 1, p, p, p, p, p, 1e-6, p, p, None), EINVAL, "prologue dtype")
    g = G(8, 16, 16, 16, 16, 16, 16, 0)
    expect(lib.di_geo_attention(ctypes.byref(g), 2, p, p, p, p, p, None), EINVAL, "attention dtype")
    expect(lib.di_node_aggregate(ctypes.byref(g), -1, p, p, p, None), EINVAL, "aggregate dtype")
    print(f"host ABI calls: {n} ok")


if __name__ == "__main__":
    main(sys.argv[1])
