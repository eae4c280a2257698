"""CPU checks of the MFMA fragment packing (csrc/common.h): emulate the gfx950 lane maps of
v_mfma_f32_16x16x32_bf16 and v_mfma_f32_16x16x4_f32 exactly as the ISA defines them and check
that a packed weight times an activation held in the row-on-lane layout equals W @ x."""
import numpy as np
import pytest
import torch

from deepinteract_amd import packing


def act_from_rows(x):
    """x [16 rows, F] -> act[lane][block][r] with feature 16*b + 4*(lane>>4) + r of row lane&15."""
    F = x.shape[1]
    act = np.zeros((64, F // 16, 4))
    for lane in range(64):
        for b in range(F // 16):
            for r in range(4):
                act[lane, b, r] = x[lane & 15, 16 * b + 4 * (lane >> 4) + r]
    return act


def rows_from_act(act):
    F = act.shape[1] * 16
    x = np.zeros((16, F))
    for lane in range(64):
        for b in range(act.shape[1]):
            for r in range(4):
                x[lane & 15, 16 * b + 4 * (lane >> 4) + r] = act[lane, b, r]
    return x


def emulate_bf16(packed, nbo, ns, act):
    out = np.zeros((64, nbo, 4))
    for s in range(ns):
        bop = np.concatenate([act[:, 2 * s, :], act[:, 2 * s + 1, :]], axis=1)  # [64, 8]
        B = np.zeros((32, 16))
        for lane in range(64):
            for j in range(8):
                B[8 * (lane >> 4) + j, lane & 15] = bop[lane, j]
        for bo in range(nbo):
            blk = packed[(bo * ns + s) * 512:(bo * ns + s + 1) * 512].reshape(64, 8)
            A = np.zeros((16, 32))
            for lane in range(64):
                for j in range(8):
                    A[lane & 15, 8 * (lane >> 4) + j] = blk[lane, j]
            D = A @ B
            for lane in range(64):
                for r in range(4):
                    out[lane, bo, r] += D[4 * (lane >> 4) + r, lane & 15]
    return out


def emulate_f32(packed, nbo, ns, act):
    out = np.zeros((64, nbo, 4))
    for s in range(ns):
        for sub in range(2):
            b = 2 * s + sub
            for r_k in range(4):
                B = np.zeros((4, 16))
                for lane in range(64):
                    B[lane >> 4, lane & 15] = act[lane, b, r_k]
                for bo in range(nbo):
                    blk = packed[(bo * ns + s) * 512:(bo * ns + s + 1) * 512].reshape(2, 64, 4)
                    A = np.zeros((16, 4))
                    for lane in range(64):
                        A[lane & 15, lane >> 4] = blk[sub, lane, r_k]
                    D = A @ B
                    for lane in range(64):
                        for r in range(4):
                            out[lane, bo, r] += D[4 * (lane >> 4) + r, lane & 15]
    return out


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("nout,kin", [(32, 64), (16, 32), (64, 128)])
def test_packed_linear_matches_dense(dtype, nout, kin):
    rng = np.random.default_rng(0)
    W = rng.integers(-4, 5, size=(nout, kin)).astype(np.float64)   # exact in bf16
    x = rng.integers(-4, 5, size=(16, kin)).astype(np.float64)
    packed = packing.pack_matrix(W, dtype)
    act = act_from_rows(x)
    out = (emulate_bf16 if dtype == "bf16" else emulate_f32)(packed, nout // 16, kin // 32, act)
    np.testing.assert_array_equal(rows_from_act(out), x @ W.T)


def test_packed32_linear_matches_dense():
    """v_mfma_f32_32x32x16_bf16 lane maps (cdna_hip_programming.md §3: A[l&31][8(l>>5)+j],
    B[8(l>>5)+j][l&31], C/D row (reg&3)+8(reg>>2)+4(l>>5), col l&31): a pack_matrix32 weight times
    an activation held as 32x32 accumulators (csrc/mfma32.h), the accumulator's registers 8t..8t+7
    of block b taken as k-step 2b+t, equals W @ x; and the chained product (output accumulator
    reused as the next B operand) too."""
    rng = np.random.default_rng(2)

    def acc_from_rows(x):  # x [32 rows, F] -> acc[lane][block][reg]
        F = x.shape[1]
        acc = np.zeros((64, F // 32, 16))
        for lane in range(64):
            for b in range(F // 32):
                for k in range(16):
                    acc[lane, b, k] = x[lane & 31, 32 * b + 8 * (k >> 2) + 4 * (lane >> 5) + (k & 3)]
        return acc

    def rows_from_acc(acc):
        x = np.zeros((32, acc.shape[1] * 32))
        for lane in range(64):
            for b in range(acc.shape[1]):
                for k in range(16):
                    x[lane & 31, 32 * b + 8 * (k >> 2) + 4 * (lane >> 5) + (k & 3)] = acc[lane, b, k]
        return x

    def emulate(packed, nbo, ns, acc):
        out = np.zeros((64, nbo, 16))
        for s in range(ns):
            bop = acc[:, s // 2, 8 * (s % 2):8 * (s % 2) + 8]  # [64, 8]
            B = np.zeros((16, 32))
            for lane in range(64):
                B[8 * (lane >> 5):8 * (lane >> 5) + 8, lane & 31] = bop[lane]
            for bo in range(nbo):
                blk = packed[(bo * ns + s) * 512:(bo * ns + s + 1) * 512].reshape(64, 8)
                A = np.zeros((32, 16))
                for lane in range(64):
                    A[lane & 31, 8 * (lane >> 5):8 * (lane >> 5) + 8] = blk[lane]
                D = A @ B
                for lane in range(64):
                    for k in range(16):
                        out[lane, bo, k] += D[(k & 3) + 8 * (k >> 2) + 4 * (lane >> 5), lane & 31]
        return out

    for nout, kin in ((32, 32), (64, 128), (128, 64)):
        W = rng.integers(-4, 5, size=(nout, kin)).astype(np.float64)
        x = rng.integers(-4, 5, size=(32, kin)).astype(np.float64)
        out = emulate(packing.pack_matrix32(W), nout // 32, kin // 16, acc_from_rows(x))
        np.testing.assert_array_equal(rows_from_acc(out), x @ W.T)
    W1 = rng.integers(-3, 4, size=(128, 64)).astype(np.float64)
    W2 = rng.integers(-3, 4, size=(64, 128)).astype(np.float64)
    x = rng.integers(-3, 4, size=(32, 64)).astype(np.float64)
    y = emulate(packing.pack_matrix32(W1), 4, 4, acc_from_rows(x))
    z = emulate(packing.pack_matrix32(W2), 2, 8, y)
    np.testing.assert_array_equal(rows_from_acc(z), x @ W1.T @ W2.T)
    # same block count and offsets as the 16-row order
    assert packing.pack_matrix32(W1).size == packing.pack_matrix(W1, "bf16").size


def test_blob_sizes_match_layout():
    from deepinteract_amd.weights import seeded_state_dict
    sd = seeded_state_dict(0, with_head=False)
    p = packing.PackedGeoT(sd, "f32")
    sizes = packing.BLOB_SIZES
    assert p.embed[0].numel() == sizes[0][0] * 512 and p.embed[1].numel() == sizes[0][1]
    assert p.init[0].numel() == sizes[1][0] * 512
    assert p.edge[0][0].numel() == sizes[2][0] * 512 and p.edge[1][0].numel() == sizes[3][0] * 512
    assert p.node[0][0].numel() == sizes[4][0] * 512 and p.node[1][0].numel() == sizes[5][0] * 512
    assert p.pos_src.shape == (2304, 128)
    pb = packing.PackedGeoT(sd, "bf16")
    assert pb.edge[0][0].dtype == torch.bfloat16
    assert pb.edge_layout == 32 and p.edge_layout == 16 and pb.init_layout == 32 and p.init_layout == 16
    assert pb.edge[0][0].numel() == sizes[2][0] * 512 and pb.edge[1][0].numel() == sizes[3][0] * 512


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("nout,kin", [(48, 113), (16, 32), (384, 128)])
def test_natural_packing_matches_dense(dtype, nout, kin):
    """di_gemm_bias_act (csrc/modules.hip): B operand read straight from x in natural k order,
    k zero-padded to 32; emulate the ISA lane maps over the packed blocks."""
    rng = np.random.default_rng(1)
    W = rng.integers(-4, 5, size=(nout, kin)).astype(np.float64)
    x = rng.integers(-4, 5, size=(16, kin)).astype(np.float64)
    packed = packing.pack_matrix_natural(W, dtype).float().numpy().astype(np.float64)
    ks = -(-kin // 32)
    xp = np.zeros((16, 32 * ks))
    xp[:, :kin] = x
    out = np.zeros((16, nout))
    for s in range(ks):
        for bo in range(nout // 16):
            blk = packed[(bo * ks + s) * 512:(bo * ks + s + 1) * 512]
            A = np.zeros((16, 32))
            if dtype == "bf16":
                b = blk.reshape(64, 8)
                for lane in range(64):
                    for j in range(8):
                        A[lane & 15, 8 * (lane >> 4) + j] = b[lane, j]
            else:
                b = blk.reshape(8, 64)
                for sub in range(8):
                    for lane in range(64):
                        A[lane & 15, 4 * sub + (lane >> 4)] = b[sub, lane]
            out[:, 16 * bo:16 * bo + 16] += (A @ xp[:, 32 * s:32 * s + 32].T).T
    np.testing.assert_array_equal(out, x @ W.T)


def test_conformation_blob_is_edge_blob_prefix():
    from deepinteract_amd.weights import seeded_state_dict
    from deepinteract_amd.config import GeoTConfig
    sd = seeded_state_dict(0, with_head=False)
    full_m, full_v = packing.edge_blob(sd, 0, False, "f32", GeoTConfig())
    conf_m, conf_v = packing.edge_blob(sd, 0, False, "f32", GeoTConfig(), conf_only=True)
    nblk, nvec = packing.BLOB_SIZES[6]
    assert conf_m.numel() == nblk * 512 and conf_v.numel() == nvec
    assert torch.equal(conf_m, full_m[:nblk * 512]) and torch.equal(conf_v, full_v[:nvec])


def test_node_count_limit_is_the_models_table_size():
    """GraphBatch enforces the model's max_num_graph_nodes (default NODE_COUNT_LIMIT=2304, the
    reference's IndexError), and a larger model (C5 class, 4096 rows) accepts longer chains."""
    import pytest
    import torch
    from deepinteract_amd.config import NODE_COUNT_LIMIT, GeoTConfig
    from deepinteract_amd.graph import GraphBatch
    from deepinteract_amd.weights import seeded_state_dict

    def gb(n, **kw):
        z = torch.zeros(n, dtype=torch.int32)
        ar = torch.arange(n, dtype=torch.int32)
        return GraphBatch(z, ar, torch.zeros(n, 4, dtype=torch.int32), None, None, [n], [n], **kw)

    assert NODE_COUNT_LIMIT == 2304
    gb(2304)
    with pytest.raises(IndexError):
        gb(2305)
    assert gb(4000, node_count_limit=4096).node_count_limit == 4096
    sd = seeded_state_dict(0, GeoTConfig(num_gnn_layers=4, knn=30, node_count_limit=4096), with_head=False)
    assert sd["gnn_module.0.init_edge_module.node_embedding.weight"].shape == (4096, 128)
    assert any(k.startswith("gnn_module.0.gt_block.3.") for k in sd)
