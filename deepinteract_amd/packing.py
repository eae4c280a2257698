"""Host-side weight preparation: BatchNorm folding, algebraic pre-multiplication and packing
into the MFMA fragment order the kernels stream (see csrc/common.h and csrc/layout.h).

Everything is computed in float64 from a reference-keyed LitGINI state dict
(deepinteract_modules.py:1478-1625 key names) and rounded once to the storage dtype.
This is model-load-time work (like a checkpoint conversion), never on the timed path.
"""
from __future__ import annotations

import numpy as np
import torch

from .config import GeoTConfig

BN_EPS = 1e-5
BLK = 512
# log2-unit SiLU (bf16 blobs only; csrc/common.h silu2): a layer whose SiLU output feeds only a
# linear layer or a gate gets its weights and bias scaled by L2E, so the kernel evaluates
# a' * rcp(1 + 2^-a') = L2E * silu(a) without the v_mul by log2(e); the consumer's weights (or
# one gate factor) are scaled by 1/L2E. Exact in real arithmetic; one bf16 rounding of the
# scaled weights.
L2E = 1.4426950408889634


def _l2e(dtype: str) -> float:
    return L2E if dtype == "bf16" else 1.0

# ---- csrc/layout.h mirror -------------------------------------------------------------------
EM_NBLK, EMV_N = 128, 384
IE_NBLK, IEV_N = 288, 384
EL_NBLK, ELV_N = 764, 2560
EL_NBLK_FINAL, ELV_N_FINAL = 572, 2048
NL_NBLK, NLV_N = 256, 768
NL_NBLK_FINAL, NLV_N_FINAL = 160, 384
EL_NBLK_CONF, ELV_N_CONF = 540, 1920
BLOB_SIZES = {0: (EM_NBLK, EMV_N), 1: (IE_NBLK, IEV_N), 2: (EL_NBLK, ELV_N),
              3: (EL_NBLK_FINAL, ELV_N_FINAL), 4: (NL_NBLK, NLV_N), 5: (NL_NBLK_FINAL, NLV_N_FINAL),
              6: (EL_NBLK_CONF, ELV_N_CONF)}


def _np(t):
    return t.detach().cpu().to(torch.float64).numpy()


def _bf16_round(x):
    return torch.from_numpy(np.asarray(x, dtype=np.float64)).to(torch.float32).to(torch.bfloat16).to(torch.float64).numpy()


def pad2(w, rows, cols):
    out = np.zeros((rows, cols), dtype=np.float64)
    out[:w.shape[0], :w.shape[1]] = w
    return out


def _pack_index(dtype: str):
    """(row, col) index arrays of one packed block, in storage order."""
    lane = np.arange(64)
    if dtype == "bf16":
        j = np.arange(8)
        row = np.broadcast_to((lane & 15)[:, None], (64, 8))
        col = 16 * (j[None, :] >> 2) + 4 * (lane[:, None] >> 4) + (j[None, :] & 3)
        return row.reshape(-1), col.reshape(-1)
    sub, r = np.arange(2), np.arange(4)
    row = np.broadcast_to((lane & 15)[None, :, None], (2, 64, 4))
    col = 16 * sub[:, None, None] + 4 * (lane[None, :, None] >> 4) + r[None, None, :]
    return row.reshape(-1), col.reshape(-1)


def pack_matrix(w, dtype: str) -> np.ndarray:
    """W [Nout, Kin] -> (Nout/16)*(Kin/32) blocks of 512 elements, block order (bo, s)."""
    w = np.asarray(w, dtype=np.float64)
    nout, kin = w.shape
    assert nout % 16 == 0 and kin % 32 == 0, (nout, kin)
    r, c = _pack_index(dtype)
    nbo, ns = nout // 16, kin // 32
    blocks = np.empty((nbo, ns, BLK), dtype=np.float64)
    for bo in range(nbo):
        for s in range(ns):
            blocks[bo, s] = w[16 * bo + r, 32 * s + c]
    return blocks.reshape(-1)


def _pack_index32():
    """(row, col) index arrays of one v_mfma_f32_32x32x16_bf16 A-fragment block (32 output rows x
    16 input features), in storage order: lane l (r = l & 31, h = l >> 5), element j holds
    W[32 ob + r][16 s + 8 (j >> 2) + 4 h + (j & 3)] -- the k order in which a 32x32 accumulator,
    converted pairwise to bf16, is the next MFMA's B operand (csrc/mfma32.h)."""
    lane = np.arange(64)
    j = np.arange(8)
    row = np.broadcast_to((lane & 31)[:, None], (64, 8))
    col = 8 * (j[None, :] >> 2) + 4 * (lane[:, None] >> 5) + (j[None, :] & 3)
    return row.reshape(-1), col.reshape(-1)


def pack_matrix32(w) -> np.ndarray:
    """W [Nout, Kin] -> (Nout/32)*(Kin/16) blocks of 512 elements, block order (ob, s): the bf16
    edge-layer blobs (di_blob_layout() == 32). Same block count as pack_matrix."""
    w = np.asarray(w, dtype=np.float64)
    nout, kin = w.shape
    assert nout % 32 == 0 and kin % 16 == 0, (nout, kin)
    r, c = _pack_index32()
    nbo, ns = nout // 32, kin // 16
    blocks = np.empty((nbo, ns, BLK), dtype=np.float64)
    for bo in range(nbo):
        for s in range(ns):
            blocks[bo, s] = w[32 * bo + r, 16 * s + c]
    return blocks.reshape(-1)


def _pack_index_natural(dtype: str):
    """Natural-k fragment order of di_gemm_bias_act (the B operand is read straight from x)."""
    lane = np.arange(64)
    if dtype == "bf16":
        j = np.arange(8)
        row = np.broadcast_to((lane & 15)[:, None], (64, 8))
        col = 8 * (lane[:, None] >> 4) + j[None, :]
        return row.reshape(-1), col.reshape(-1)
    sub = np.arange(8)
    row = np.broadcast_to((lane & 15)[None, :], (8, 64))
    col = 4 * sub[:, None] + (lane[None, :] >> 4)
    return row.reshape(-1), col.reshape(-1)


def pack_matrix_natural(w, dtype: str) -> torch.Tensor:
    """W [Nout, Kin] (Nout % 16 == 0; Kin zero-padded to a multiple of 32) -> packed blocks in
    the storage dtype, block order (bo, s), for di_gemm_bias_act."""
    w = np.asarray(w, dtype=np.float64)
    nout, kin = w.shape
    assert nout % 16 == 0, nout
    w = pad2(w, nout, -(-kin // 32) * 32)
    r, c = _pack_index_natural(dtype)
    nbo, ns = nout // 16, w.shape[1] // 32
    blocks = np.empty((nbo, ns, BLK), dtype=np.float64)
    for bo in range(nbo):
        for s in range(ns):
            blocks[bo, s] = w[16 * bo + r, 32 * s + c]
    t = torch.from_numpy(blocks.reshape(-1)).to(torch.float32)
    return t.to(torch.bfloat16) if dtype == "bf16" else t


def bn_affine(sd, name):
    g, b = _np(sd[f"{name}.weight"]), _np(sd[f"{name}.bias"])
    m, v = _np(sd[f"{name}.running_mean"]), _np(sd[f"{name}.running_var"])
    s = g / np.sqrt(v + BN_EPS)
    return s, b - m * s


def lin(sd, name):
    w = _np(sd[f"{name}.weight"])
    b = _np(sd[f"{name}.bias"]) if f"{name}.bias" in sd else np.zeros(w.shape[0])
    return w, b


def fold_bn_before(w, b, s, t):
    """Linear(BN(x)) = (W diag s) x + (W t + b)."""
    return w * s[None, :], w @ t + b


def fold_bn_after(w, b, s, t):
    """BN(Linear(x)) = (diag s W) x + (s b + t)."""
    return w * s[:, None], s * b + t


class BlobBuilder:
    def __init__(self, dtype: str, nblk: int, nvec: int, layout: int = 16):
        assert layout in (16, 32) and (layout == 16 or dtype == "bf16"), (dtype, layout)
        self.dtype, self.nblk, self.nvec, self.layout = dtype, nblk, nvec, layout
        self.mat = np.zeros(nblk * BLK, dtype=np.float64)
        self.vec = np.zeros(nvec, dtype=np.float64)
        self.used = np.zeros(nblk, dtype=bool)

    def put(self, blk_off: int, w):
        p = pack_matrix32(w) if self.layout == 32 else pack_matrix(w, self.dtype)
        n = p.size // BLK
        assert blk_off + n <= self.nblk, (blk_off, n, self.nblk)
        assert not self.used[blk_off:blk_off + n].any(), blk_off
        self.used[blk_off:blk_off + n] = True
        self.mat[blk_off * BLK:(blk_off + n) * BLK] = p

    def putv(self, off: int, v):
        v = np.asarray(v, dtype=np.float64).reshape(-1)
        assert off + v.size <= self.nvec
        self.vec[off:off + v.size] = v

    def finish(self):
        assert self.used.all(), np.nonzero(~self.used)[0][:8]
        t = torch.from_numpy(self.mat).to(torch.float32)
        if self.dtype == "bf16":
            t = t.to(torch.bfloat16)
        return t, torch.from_numpy(self.vec).to(torch.float32)


# ---- per-kernel blobs ---------------------------------------------------------------------------
def _qkv(sd, li):
    p = f"gnn_module.0.gt_block.{li}"
    s, t = bn_affine(sd, f"{p}.batch_norm1_node_feats")
    out = []
    for q in ("Q", "K", "V"):
        w, b = lin(sd, f"{p}.mha_module.{q}")
        out.append(fold_bn_before(w, b, s, t))
    return out


def embed_blob(sd, dtype):
    bb = BlobBuilder(dtype, EM_NBLK, EMV_N)
    bb.put(0, pad2(_np(sd["node_in_embedding.weight"]), 128, 128))
    for i, (w, b) in enumerate(_qkv(sd, 0)):
        bb.put(32 + 32 * i, w)
        bb.putv(128 * i, b)
    return bb.finish()


GEO_COLS = {"edge_messages": (0, 2), "dist": (2, 20), "dir": (20, 23), "orient": (23, 27), "amide": (27, 28)}
GEO_ORDER = ("edge_messages", "dist", "dir", "orient", "amide")


def _geo_rows(w, kind):
    """[out, k_kind] weight placed on its columns of the 28 (padded 32) edge features."""
    lo, hi = GEO_COLS[kind]
    full = np.zeros((w.shape[0], 32))
    full[:, lo:hi] = w
    return full


def init_blob(sd, dtype, p="gnn_module.0.init_edge_module",
              nbr="gnn_module.0.gt_block.0.conformation_module.nbr_linear", layout=16):
    """nbr=None: no following layer (standalone InitEdgeModule): the fused silu(nbr_linear)
    output is computed with zero weights and ignored. layout: fragment order (16, or 32 for the
    bf16 32x32x16 InitEdge kernels)."""
    bb = BlobBuilder(dtype, IE_NBLK, IEV_N, layout)
    sc = _l2e(dtype)  # log2-unit SiLU: geometric projections, combined logits and gates (silu2)
    wc0 = _np(sd[f"{p}.combined_linear_0.weight"])  # [128, 896]
    for t, kind in enumerate(GEO_ORDER):
        w0 = _np(sd[f"{p}.{kind}_linear_0.weight"])
        if t == 0:
            # edge_messages_linear_0 has no activation before combined_linear_0 (:237-241), so its
            # slice of combined_linear_0 collapses with it into ONE [128, 2] map of the two message
            # columns (pos_enc, weight): 8 blocks / 8 MFMAs instead of 40; blocks 8..39 stay zero
            bb.put(0, _geo_rows(wc0[:, 256:384] @ w0, kind) * sc)
            bb.put(8, np.zeros((128, 128)))  # unused (layout kept)
        else:
            # silu2(sc * W_t0 g) = sc * silu(W_t0 g), consumed by wc0 (x 1/sc), accumulated into
            # sc * acc (x sc): net 1
            bb.put(40 * t, _geo_rows(w0, kind) * sc)
            bb.put(40 * t + 8, wc0[:, 256 + 128 * t: 384 + 128 * t])
        bb.put(200 + 8 * t, _geo_rows(_np(sd[f"{p}.{kind}_linear_1.weight"]), kind) * sc)  # gs' = sc * gs
    # silu2(sc * acc) * (sc * gs) = sc^2 * (silu(acc) * gs)
    bb.put(240, pad2(_np(sd[f"{p}.combined_linear_1.weight"]), 32, 128) / (sc * sc))
    bb.put(248, pad2(_np(sd[f"{p}.combined_linear_2.weight"]), 128, 32))
    w, b = lin(sd, nbr) if nbr else (np.zeros((128, 128)), np.zeros(128))
    bb.put(256, w)
    bb.putv(0, b)
    # DI_GRAPH_GEO_REF batches (orientation columns = (0, 0, 0, 1) on every edge): the orientation
    # terms are per-model constants (deepinteract_modules.py:226, :243), in the kernel's units (x sc)
    silu = lambda x: x / (1.0 + np.exp(-x))  # noqa: E731
    t_or = GEO_ORDER.index("orient")
    o0 = _np(sd[f"{p}.orient_linear_0.weight"])[:, 3]
    o1 = _np(sd[f"{p}.orient_linear_1.weight"])[:, 3]
    orc = (wc0[:, 256 + 128 * t_or: 384 + 128 * t_or] @ silu(o0)) * sc
    bb.putv(128, orc)
    bb.putv(256, silu(o1) * sc)
    if layout == 32:
        # the 32x32 kernels take the orientation constant through the collapsed message map: columns
        # 28 / 29 (padding of the 28 edge features) hold it as a bf16 hi + lo pair, and the GEO_REF
        # kernels set geometric features 28 / 29 to 1 (the general path leaves them 0); every other
        # geometric matrix is zero in those columns
        hi = _bf16_round(orc)
        t0 = _geo_rows(wc0[:, 256:384] @ _np(sd[f"{p}.edge_messages_linear_0.weight"]), "edge_messages") * sc
        t0[:, 28] = hi
        t0[:, 29] = orc - hi
        bb.used[0:8] = False
        bb.put(0, t0)
    mat, vec = bb.finish()
    emb = _np(sd[f"{p}.node_embedding.weight"])
    pos_src = torch.from_numpy(emb @ wc0[:, 0:128].T * sc).to(torch.float32)
    pos_dst = torch.from_numpy(emb @ wc0[:, 128:256].T * sc).to(torch.float32)
    return mat, vec, pos_src, pos_dst


def edge_blob(sd, li, final, dtype, cfg: GeoTConfig, conf_only=False, c=None, layout=16):
    """final: kind 3, else kind 2; conf_only: kind 6 (ConformationModule alone, key prefix c).
    layout: the fragment order of the matrices (16, or 32 for the bf16 32x32x16 edge kernel)."""
    p = f"gnn_module.0.gt_block.{li}"
    c = c or f"{p}.conformation_module"
    if conf_only:
        bb = BlobBuilder(dtype, EL_NBLK_CONF, ELV_N_CONF, layout)
    else:
        bb = BlobBuilder(dtype, EL_NBLK_FINAL if final else EL_NBLK, ELV_N_FINAL if final else ELV_N, layout)
    sc = _l2e(dtype)  # log2-unit SiLU: downward_proj, ResBlock layers 0-1, edge FFN (silu2)
    two = lambda a, b: _np(sd[f"{c}.{a}.weight"]) @ _np(sd[f"{c}.{b}.weight"])  # noqa: E731
    mg = np.zeros((320, 32))
    mg[0:128] = _geo_rows(two("dist_linear_1", "dist_linear_0"), "dist")
    mg[128:192] = _geo_rows(two("dir_linear_1", "dir_linear_0"), "dir") / sc  # gate x 1/sc
    mg[192:256] = _geo_rows(two("orient_linear_1", "orient_linear_0"), "orient")
    mg[256:320] = _geo_rows(two("amide_linear_1", "amide_linear_0"), "amide")
    fg = np.zeros((128, 32))
    for kind, name in (("dist", "final_dist_linear"), ("dir", "final_dir_linear"),
                       ("orient", "final_orient_linear"), ("amide", "final_amide_linear")):
        fg += _geo_rows(_np(sd[f"{c}.{name}.weight"]), kind)
    bb.put(0, mg)
    bb.put(20, _np(sd[f"{c}.downward_proj.weight"]) * sc)
    bb.put(36, _np(sd[f"{c}.upward_proj.weight"]) * sc)  # silu2, ln2 folded into the bias add
    w, b = lin(sd, f"{c}.orig_msg_linear")
    bb.put(52, w)
    bb.putv(0, b)
    i = 0
    for kind in ("pre_res_blocks", "post_res_blocks"):
        for rb in range(2):
            r = f"{c}.{kind}.{rb}.res_block"
            s, t = bn_affine(sd, f"{r}.1")  # one BatchNorm instance reused 3x (:468-479)
            for l in (0, 3, 6):
                w, b = lin(sd, f"{r}.{l}")
                w, b = fold_bn_after(w, b, s, t)
                w_in = 1.0 if l == 0 else 1.0 / sc   # input in log2 units after layers 0 and 3
                w_out = sc                           # every layer feeds silu2 (layer 6: ln2 in the residual fma)
                bb.put(84 + 32 * i, w * (w_in * w_out))
                bb.putv(128 + 128 * i, b * w_out)
                i += 1
    w, b = lin(sd, f"{c}.res_connect_linear")  # silu2, ln2 folded into the residual fma
    bb.put(468, w * sc)
    bb.putv(1664, b * sc)
    w, b = lin(sd, f"{c}.final_linear")  # silu2, ln2 folded into the residual fma
    bb.put(500, w * sc)
    bb.putv(1792, b * sc)
    bb.put(532, fg)
    if conf_only:
        return bb.finish()
    s, t = bn_affine(sd, f"{p}.batch_norm1_edge_feats")
    w, b = fold_bn_before(*lin(sd, f"{p}.mha_module.edge_feats_projection"), s, t)
    bb.put(540, w)
    bb.putv(1920, b)
    if not final:
        w, b = lin(sd, f"{p}.O_edge_feats")
        bb.put(572, w)
        bb.putv(2048, b)
        s, t = bn_affine(sd, f"{p}.batch_norm2_edge_feats")
        w1, b1 = fold_bn_before(*lin(sd, f"{p}.edge_feats_MLP.0"), s, t)
        bb.put(604, w1[:128] * sc)
        bb.put(636, w1[128:] * sc)
        bb.putv(2176, b1 * sc)
        w2 = _np(sd[f"{p}.edge_feats_MLP.3.weight"]) / sc
        bb.put(668, w2[:, :128])
        bb.put(700, w2[:, 128:])
        w, b = lin(sd, f"gnn_module.0.gt_block.{li + 1}.conformation_module.nbr_linear")
        bb.put(732, w)
        bb.putv(2432, b)
    return bb.finish()


def node_blob(sd, li, final, dtype):
    p = f"gnn_module.0.gt_block.{li}"
    bb = BlobBuilder(dtype, NL_NBLK_FINAL if final else NL_NBLK, NLV_N_FINAL if final else NLV_N)
    w, b = lin(sd, f"{p}.O_node_feats")
    bb.put(0, w)
    bb.putv(0, b)
    s, t = bn_affine(sd, f"{p}.batch_norm2_node_feats")
    sc = _l2e(dtype)  # log2-unit SiLU in the node FFN (silu2)
    w1, b1 = fold_bn_before(*lin(sd, f"{p}.node_feats_MLP.0"), s, t)
    bb.put(32, w1[:128] * sc)
    bb.put(64, w1[128:] * sc)
    bb.putv(128, b1 * sc)
    w2 = _np(sd[f"{p}.node_feats_MLP.3.weight"]) / sc
    bb.put(96, w2[:, :128])
    bb.put(128, w2[:, 128:])
    if not final:
        for i, (w, b) in enumerate(_qkv(sd, li + 1)):
            bb.put(160 + 32 * i, w)
            bb.putv(384 + 128 * i, b)
    return bb.finish()


# fragment order of the edge-layer and InitEdge blobs the shipped library expects (di_blob_layout(1 / 2 / 3, dtype))
EDGE_LAYOUT_DEFAULT = {"bf16": 32, "f32": 16}


class PackedGeoT:
    """All device-ready weight blobs of one DGLGeometricTransformer (+ node_in_embedding)."""

    def __init__(self, sd, dtype: str = "f32", cfg: GeoTConfig = GeoTConfig(), device="cpu", edge_layout=None,
                 init_layout=None):
        """edge_layout / init_layout: fragment order of the edge-layer / InitEdge blobs (the library's
        di_blob_layout(2 / 1, dt)); None: this build's default (32 for bf16, 16 for fp32)."""
        assert dtype in ("f32", "bf16")
        if edge_layout is None:
            edge_layout = EDGE_LAYOUT_DEFAULT[dtype]
        if init_layout is None:
            init_layout = EDGE_LAYOUT_DEFAULT[dtype]
        self.dtype, self.cfg, self.edge_layout, self.init_layout = dtype, cfg, edge_layout, init_layout
        L = cfg.num_gnn_layers
        dev = torch.device(device)
        mv = lambda pair: tuple(x.to(dev).contiguous() for x in pair)  # noqa: E731
        self.embed = mv(embed_blob(sd, dtype))
        im, iv, ps, pd = init_blob(sd, dtype, layout=init_layout)
        self.init = mv((im, iv))
        self.pos_src, self.pos_dst = ps.to(dev).contiguous(), pd.to(dev).contiguous()
        self.edge = [mv(edge_blob(sd, li, li == L - 1, dtype, cfg, layout=edge_layout)) for li in range(L)]
        self.node = [mv(node_blob(sd, li, li == L - 1, dtype)) for li in range(L)]

    @property
    def num_layers(self):
        return len(self.edge)
