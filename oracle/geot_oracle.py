"""ORACLE — CPU fp32 restatement of DeepInteract's GeoT hot path. TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline. The product package
``deepinteract_amd`` never imports it.

This is an op-for-op restatement (plain PyTorch on CPU, fp32) of the reference's algorithm,
written DGL-style so that its cost profile is the reference's: full-edge gathers per
``apply_edges``, the [E,N] ``i_all`` gather in InitEdge, ``index_add`` for
``send_and_recv``, and ``repeat_interleave`` + ``cat`` for the pair tensor. Each function
cites the reference file:line it restates (paths relative to ``project/utils/`` unless
stated).

Pinning: ``tests/test_oracle_golden.py`` checks this oracle against golden vectors produced
by the reference's own, unmodified Python modules (``tests/golden/make_golden.py``).
DGL 0.6 semantics used here (kNN edge order, in_edges order) are restated in the
[DGL-ASSUMPTION] comments; they are the same ones ``tests/golden/refshim.py`` restates.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

KNN = 20
NB = 2  # geo_nbrhd_size (lit_model_predict.py:156)
NUM_RBF = 18
H = 128
HEADS = 4
DH = 32
BN_EPS = 1e-5
IN_EPS = 1e-6


# =========================================================================================
# Graph builder (deepinteract_utils.py:386-555, graph_utils.py:69-110,
#                protein_feature_utils.py:63-377)
# =========================================================================================
def pairwise_squared_distance(x):
    """dgl.nn.pytorch.pairwise_squared_distance (graph_utils.py:7,108): expansion formula."""
    x2s = torch.sum(x * x, -1, keepdim=True)
    return x2s + x2s.transpose(-1, -2) - 2 * x @ x.transpose(-1, -2)


def knn(ca, k=KNN):
    """graph_utils.py:107-108. [DGL-ASSUMPTION, DGL 0.6 _knn_graph_blas] edge e = i*k + r has
    src = idx[i, r], dst = i. Returns (idx [N,k] i64, d2 [N,k] f32 sorted ascending)."""
    d = pairwise_squared_distance(ca)
    vals, idx = torch.topk(d, k, dim=1, largest=False)
    return idx, vals


def _normalize(x, dim=-1):
    return F.normalize(x, dim=dim)


def dihedrals(X, eps=1e-7):
    """protein_feature_utils.py:276-320 (X [1,N,4,3]) -> [1,N,6] cos/sin of phi, psi, omega."""
    X = X[:, :, :3, :].reshape(X.shape[0], 3 * X.shape[1], 3)
    dX = X[:, 1:, :] - X[:, :-1, :]
    U = _normalize(dX)
    u_2, u_1, u_0 = U[:, :-2, :], U[:, 1:-1, :], U[:, 2:, :]
    n_2 = _normalize(torch.cross(u_2, u_1, dim=-1))
    n_1 = _normalize(torch.cross(u_1, u_0, dim=-1))
    cosD = torch.clamp((n_2 * n_1).sum(-1), -1 + eps, 1 - eps)
    D = torch.sign((u_2 * n_1).sum(-1)) * torch.acos(cosD)
    D = F.pad(D, (1, 2), 'constant', 0)
    D = D.view((D.size(0), int(D.size(1) / 3), 3))
    return torch.cat((torch.cos(D), torch.sin(D)), 2)


def rbf(d2, num_rbf=NUM_RBF):
    """protein_feature_utils.py:82-101 — RBF of SQUARED distances."""
    mu = torch.linspace(0., 20., num_rbf).view([1, 1, 1, -1])
    sigma = 20. / num_rbf
    return torch.exp(-((d2.unsqueeze(-1) - mu) / sigma) ** 2)


def _quaternions(R):
    """protein_feature_utils.py:104-149."""
    diag = torch.diagonal(R, dim1=-2, dim2=-1)
    Rxx, Ryy, Rzz = diag.unbind(-1)
    mag = 0.5 * torch.sqrt(torch.abs(1 + torch.stack([Rxx - Ryy - Rzz, -Rxx + Ryy - Rzz, -Rxx - Ryy + Rzz], -1)))
    signs = torch.sign(torch.stack([R[..., 2, 1] - R[..., 1, 2], R[..., 0, 2] - R[..., 2, 0],
                                    R[..., 1, 0] - R[..., 0, 1]], -1))
    w = torch.sqrt(F.relu(1 + diag.sum(-1, keepdim=True))) / 2.
    return _normalize(torch.cat((signs * mag, w), -1))


def orientations(Xca, E_idx):
    """protein_feature_utils.py:201-273 (O_features only): dU (3) + quaternion (4)."""
    dX = Xca[:, 1:, :] - Xca[:, :-1, :]
    U = _normalize(dX)
    u_2, u_1 = U[:, :-2, :], U[:, 1:-1, :]
    n_2 = _normalize(torch.cross(u_2, u_1, dim=-1))
    o_1 = _normalize(u_2 - u_1)
    O = torch.stack((o_1, n_2, torch.cross(o_1, n_2, dim=-1)), 2)
    O = O.view(list(O.shape[:2]) + [9])
    O = F.pad(O, (0, 0, 1, 2), 'constant', 0)
    B, N, K = E_idx.shape
    flat = E_idx.view(B, -1)
    O_nb = torch.gather(O, 1, flat.unsqueeze(-1).expand(-1, -1, 9)).view(B, N, K, 9)
    X_nb = torch.gather(Xca, 1, flat.unsqueeze(-1).expand(-1, -1, 3)).view(B, N, K, 3)
    O = O.view(B, N, 3, 3)
    O_nb = O_nb.view(B, N, K, 3, 3)
    dXn = X_nb - Xca.unsqueeze(-2)
    dU = _normalize(torch.matmul(O.unsqueeze(2), dXn.unsqueeze(-1)).squeeze(-1))
    R = torch.matmul(O.unsqueeze(2).transpose(-1, -2), O_nb)
    return torch.cat((dU, _quaternions(R)), -1)


def minmax(t):
    """deepinteract_utils.py:79-84 (element-wise (v - min)/(max - min), fp32)."""
    mn, mx = t.min(), t.max()
    return (t - mn) / (mx - mn)


def build_graph(chain, k=KNN, nb=NB, seed=None, generator=None):
    """convert_df_to_dgl_graph (deepinteract_utils.py:386-555) restated on arrays.

    chain: dict with backbone [N,4,3], amide_norm [N,3], dips [N,106] (numpy or torch).
    Neighbour ids use torch.randperm exactly as the reference loop does (:539-546) —
    E calls for the src side then E calls for the dst side — so the same seed gives the same
    ids. [DGL-ASSUMPTION] in_edges(v) lists v's in-edges in edge-id order, i.e. v*k..v*k+k-1.
    """
    bb = torch.as_tensor(np.asarray(chain["backbone"]), dtype=torch.float32)
    N = bb.shape[0]
    ca = bb[:, 1, :].contiguous()
    idx, d2 = knn(ca, k)
    src = idx.reshape(-1)
    dst = torch.arange(N).repeat_interleave(k)
    # geometric features (:460-490); mask of finite coords is all-true for complete backbones
    X = bb.reshape(1, N, 4, 3)
    E_idx = dst.reshape(1, N, k)  # ':476 edges_transformed = edges[1]'
    node_geo = dihedrals(X)[0]
    edge_rbf = rbf(d2.reshape(1, N, k))[0].reshape(-1, NUM_RBF)
    edge_ori = orientations(X[:, :, 1, :], E_idx)[0].reshape(-1, 7)
    # node features (:494-498)
    pos = minmax(torch.arange(N)).to(torch.float32).reshape(-1, 1) if N > 1 else torch.zeros(1, 1)
    dips = torch.as_tensor(np.asarray(chain["dips"]), dtype=torch.float32)
    node_f = torch.cat((pos, node_geo, dips), 1)
    # edge features (:504-530)
    pos_e = torch.sin((src - dst).float()).reshape(-1, 1)
    w = minmax(torch.sum((ca[src] - ca[dst]) ** 2, 1)).reshape(-1, 1)
    am = torch.as_tensor(np.asarray(chain["amide_norm"]), dtype=torch.float32)
    v1, v2 = am[dst], am[src]
    cosang = (v1 * v2).sum(-1) / (torch.linalg.norm(v1, dim=-1) * torch.linalg.norm(v2, dim=-1))
    ang = torch.nan_to_num(torch.acos(cosang), nan=0.0)
    ang = torch.nan_to_num(minmax(ang), nan=0.0).reshape(-1, 1)
    edge_f = torch.cat((pos_e, w, edge_rbf, edge_ori[:, :3], edge_ori[:, 3:], ang), 1)
    # neighbour edge ids (:534-553)
    if generator is None:
        generator = torch.Generator()
        generator.manual_seed(0 if seed is None else seed)
    E = N * k
    ps = torch.stack([torch.randperm(k, generator=generator) for _ in range(E)])[:, :nb]
    pd = torch.stack([torch.randperm(k, generator=generator) for _ in range(E)])[:, :nb]
    src_nbr = src.reshape(-1, 1) * k + ps
    dst_nbr = dst.reshape(-1, 1) * k + pd
    return {
        "num_nodes": N, "src": src, "dst": dst, "idx": idx, "d2": d2,
        "node_f": node_f, "edge_f": edge_f, "src_nbr": src_nbr, "dst_nbr": dst_nbr,
    }


# =========================================================================================
# GeoT forward (deepinteract_modules.py)
# =========================================================================================
def _lin(x, sd, name):
    """nn.Linear: bias applied iff the state dict holds one for this layer."""
    return F.linear(x, sd[f"{name}.weight"], sd.get(f"{name}.bias"))


def _bn(x, sd, name):
    return F.batch_norm(x, sd[f"{name}.running_mean"], sd[f"{name}.running_var"],
                        sd[f"{name}.weight"], sd[f"{name}.bias"], False, 0.0, BN_EPS)


def _geo(G):
    """get_geo_feats_from_edges (deepinteract_utils.py:70-76)."""
    return G[:, 2:20], G[:, 20:23], G[:, 23:27], G[:, 27]


def init_edge(sd, g, edge_f):
    """InitEdgeModule (deepinteract_modules.py:198-264), incl. the [E,N] i_all gather."""
    p = "gnn_module.0.init_edge_module"
    silu = F.silu
    N, src, dst = g["num_nodes"], g["src"], g["dst"]
    nodes = torch.arange(N)
    i_all = torch.cat((nodes, nodes.repeat(N - 1))).reshape(N, N)           # :261
    node_indices = i_all[src][0]                                            # :209 ([E,N] gather)
    node_feats = F.embedding(node_indices, sd[f"{p}.node_embedding.weight"])
    s_nf, d_nf = node_feats[nodes[src]], node_feats[nodes[dst]]            # :211
    m = torch.cat((edge_f[:, 0].reshape(-1, 1), edge_f[:, 1].reshape(-1, 1)), 1)
    dist, dirf, ori, am = _geo(edge_f)
    am = am.reshape(-1, 1)
    em0 = _lin(m, sd, f"{p}.edge_messages_linear_0")
    c = silu(_lin(torch.cat([s_nf, d_nf, em0,
                             silu(_lin(dist, sd, f"{p}.dist_linear_0")),
                             silu(_lin(dirf, sd, f"{p}.dir_linear_0")),
                             silu(_lin(ori, sd, f"{p}.orient_linear_0")),
                             silu(_lin(am, sd, f"{p}.amide_linear_0"))], 1), sd, f"{p}.combined_linear_0"))
    s = (_lin(m, sd, f"{p}.edge_messages_linear_1") * c
         + silu(_lin(dist, sd, f"{p}.dist_linear_1")) * c
         + silu(_lin(dirf, sd, f"{p}.dir_linear_1")) * c
         + silu(_lin(ori, sd, f"{p}.orient_linear_1")) * c
         + silu(_lin(am, sd, f"{p}.amide_linear_1")) * c)
    return _lin(_lin(s, sd, f"{p}.combined_linear_1"), sd, f"{p}.combined_linear_2")


def _resblock(sd, p, x):
    """ResBlock (deepinteract_modules.py:458-497): one BN instance reused 3x."""
    y = x
    for i in (0, 3, 6):
        y = F.silu(_bn(_lin(y, sd, f"{p}.res_block.{i}"), sd, f"{p}.res_block.1"))
    return x + y


def conformation(sd, p, g, F_cur, G):
    """ConformationModule (deepinteract_modules.py:373-455)."""
    silu = F.silu
    src_ids, dst_ids = g["src_nbr"].permute(1, 0), g["dst_nbr"].permute(1, 0)
    nbr = torch.cat((F_cur[src_ids], F_cur[dst_ids]))                       # [4,E,H]
    nbr = silu(_lin(nbr, sd, f"{p}.nbr_linear"))
    dist, dirf, ori, am = _geo(G)
    am = am.reshape(-1, 1)
    nbr = nbr * _lin(_lin(dist, sd, f"{p}.dist_linear_0"), sd, f"{p}.dist_linear_1")
    nbr = silu(_lin(nbr, sd, f"{p}.downward_proj"))
    nbr = nbr * _lin(_lin(dirf, sd, f"{p}.dir_linear_0"), sd, f"{p}.dir_linear_1")
    nbr = nbr * _lin(_lin(ori, sd, f"{p}.orient_linear_0"), sd, f"{p}.orient_linear_1")
    nbr = nbr * _lin(_lin(am, sd, f"{p}.amide_linear_0"), sd, f"{p}.amide_linear_1")
    nbr = silu(_lin(torch.sum(nbr, dim=0), sd, f"{p}.upward_proj"))
    x = _lin(F_cur, sd, f"{p}.orig_msg_linear") + nbr
    for b in range(2):
        x = _resblock(sd, f"{p}.pre_res_blocks.{b}", x)
    x = F_cur + silu(_lin(x, sd, f"{p}.res_connect_linear"))
    for b in range(2):
        x = _resblock(sd, f"{p}.post_res_blocks.{b}", x)
    gsum = (_lin(dist, sd, f"{p}.final_dist_linear") * x + _lin(dirf, sd, f"{p}.final_dir_linear") * x
            + _lin(ori, sd, f"{p}.final_orient_linear") * x + _lin(am, sd, f"{p}.final_amide_linear") * x)
    return F_cur + silu(_lin(gsum, sd, f"{p}.final_linear"))


def mha(sd, p, g, node, edge, update_edge_feats):
    """MultiHeadGeometricAttentionLayer (deepinteract_modules.py:76-121) with the edge UDFs
    of graph_utils.py:21-63 and DGL send_and_recv(u_mul_e/copy_e, sum) as index_add."""
    src, dst, N = g["src"], g["dst"], g["num_nodes"]
    Q = _lin(node, sd, f"{p}.Q").view(-1, HEADS, DH)
    K = _lin(node, sd, f"{p}.K").view(-1, HEADS, DH)
    V = _lin(node, sd, f"{p}.V").view(-1, HEADS, DH)
    P = _lin(edge, sd, f"{p}.edge_feats_projection").view(-1, HEADS, DH)
    score = K[src] * Q[dst]                                                 # src_dot_dst
    score = (score / np.sqrt(DH)).clamp(-5.0, 5.0)                          # scaling
    score = score * P                                                       # imp_exp_attn
    e_out = score if update_edge_feats else None                            # out_edge_features
    score = torch.exp(score.sum(-1, keepdim=True).clamp(-5.0, 5.0))         # exp
    wV = torch.zeros(N, HEADS, DH).index_add_(0, dst, V[src] * score)      # u_mul_e, sum
    z = torch.zeros(N, HEADS, 1).index_add_(0, dst, score)                  # copy_e, sum
    h = wV / (z + torch.full_like(z, 1e-6))
    return h, e_out


def gt_layer(sd, li, g, node, edge, G, final):
    """GeometricTransformerModule.run_gt_layer (:669-727) / Final... (:892-946), eval."""
    p = f"gnn_module.0.gt_block.{li}"
    n1, e1 = node, edge
    c = conformation(sd, f"{p}.conformation_module", g, edge, G)
    n_b = _bn(node, sd, f"{p}.batch_norm1_node_feats")
    e_b = _bn(c, sd, f"{p}.batch_norm1_edge_feats")
    h, e_out = mha(sd, f"{p}.mha_module", g, n_b, e_b, update_edge_feats=not final)
    n = n1 + _lin(h.reshape(-1, H), sd, f"{p}.O_node_feats")
    n = n + _lin(F.silu(_lin(_bn(n, sd, f"{p}.batch_norm2_node_feats"), sd, f"{p}.node_feats_MLP.0")),
                 sd, f"{p}.node_feats_MLP.3")
    if final:
        return n, None, c
    e = e1 + _lin(e_out.reshape(-1, H), sd, f"{p}.O_edge_feats")
    e = e + _lin(F.silu(_lin(_bn(e, sd, f"{p}.batch_norm2_edge_feats"), sd, f"{p}.edge_feats_MLP.0")),
                 sd, f"{p}.edge_feats_MLP.3")
    return n, e, c


def geot_forward(sd, g, num_layers=2, return_intermediates=False):
    """LitGINI.gnn_forward (:1660-1679) + DGLGeometricTransformer.forward (:1426-1466)
    for ONE chain. Returns node [N,128], edge [E,128] (last intermediate layer's edges, :1457)."""
    inter = {}
    G = g["edge_f"]
    node = _lin(g["node_f"], sd, "node_in_embedding")
    edge = init_edge(sd, g, G)
    inter["node_emb"], inter["init_edge"] = node, edge
    for li in range(num_layers - 1):
        node, edge, c = gt_layer(sd, li, g, node, edge, G, final=False)
        inter[f"conf{li}"], inter[f"node{li}"], inter[f"edge{li}"] = c, node, edge
    node, _, c = gt_layer(sd, num_layers - 1, g, node, edge, G, final=True)
    inter[f"conf{num_layers - 1}"] = c
    if return_intermediates:
        return node, edge, inter
    return node, edge


def pair_tensor(h1, h2):
    """construct_interact_tensor, pad=False (deepinteract_utils.py:158-172)."""
    L1, L2 = h1.shape[0], h2.shape[0]
    xa, xb = h1.permute(1, 0).unsqueeze(0), h2.permute(1, 0).unsqueeze(0)
    return torch.cat((torch.repeat_interleave(xa.unsqueeze(3), repeats=L2, dim=3),
                      torch.repeat_interleave(xb.unsqueeze(2), repeats=L1, dim=2)), dim=1)


# =========================================================================================
# Head (stays on PyTorch in the product; restated here for logits parity)
# =========================================================================================
def _conv(x, sd, name, dilation=1, padding=0):
    return F.conv2d(x, sd[f"{name}.weight"], sd[f"{name}.bias"], padding=padding, dilation=dilation)


def _inorm(x, sd, name):
    return F.instance_norm(x, weight=sd[f"{name}.weight"], bias=sd[f"{name}.bias"], eps=IN_EPS)


def _se(x, sd, name):
    """SEBlock (deepinteract_modules.py:954-970)."""
    s = torch.mean(x.reshape(x.shape[0], x.shape[1], -1), dim=-1)
    s = F.relu(_lin(s, sd, f"{name}.linear1"))
    s = torch.sigmoid(F.relu(_lin(s, sd, f"{name}.linear2")))
    return torch.einsum('bcij,bc->bcij', x, s)


def _resnet(x, sd, prefix, mname, chunks, inorm, extra):
    """ResNet.forward (deepinteract_modules.py:1051-1106)."""
    x = _conv(x, sd, f"{prefix}.resnet_{mname}_init_proj")
    blocks = [(f"{i}_{d}", d) for i in range(chunks) for d in (1, 2, 4, 8)]
    if extra:
        blocks += [("extra0", 1), ("extra1", 1)]
    for b, d in blocks:
        r = f"{prefix}.resnet_{mname}_{b}"
        res = x
        if inorm:
            x = _inorm(x, sd, f"{r}_inorm_1")
        x = _conv(F.elu(x), sd, f"{r}_conv2d_1")
        if inorm:
            x = _inorm(x, sd, f"{r}_inorm_2")
        x = _conv(F.elu(x), sd, f"{r}_conv2d_2", dilation=d, padding=d)
        if inorm:
            x = _inorm(x, sd, f"{r}_inorm_3")
        x = _conv(F.elu(x), sd, f"{r}_conv2d_3")
        x = _se(x, sd, f"{r}_se_block") + res
    return x


def head_prologue(sd, t):
    """First line of ResNet2DInputWithOptAttention.forward (deepinteract_modules.py:1231-1232):
    ELU(inorm_1(conv2d_1(t))) on the materialised pair tensor t."""
    p = "interact_module"
    return F.elu(_inorm(_conv(t, sd, f"{p}.conv2d_1"), sd, f"{p}.inorm_1"))


def head_forward(sd, t, num_chunks=14):
    """ResNet2DInputWithOptAttention.forward (deepinteract_modules.py:1228-1248), no attention."""
    p = "interact_module"
    x = head_prologue(sd, t)
    x = F.elu(_resnet(x, sd, f"{p}.base_resnet", "base_resnet", num_chunks, True, False))
    x = F.elu(_resnet(x, sd, f"{p}.phase2_resnet", "bin_resnet", 1, False, True))
    return _conv(x, sd, f"{p}.phase2_conv")


def contact_probs(logits):
    """lit_model_predict.py:236-239: softmax over classes, positive class -> [L1,L2]."""
    L1, L2 = logits.shape[-2:]
    flat = torch.flatten(logits.squeeze(0), start_dim=1).transpose(1, 0)
    return torch.softmax(flat, dim=1)[:, 1].reshape(L1, L2)


def predict(sd, g1, g2, num_layers=2, num_chunks=14):
    """LitGINI.shared_step (:1687-1745) for one complex -> (logits, n1, e1, n2, e2)."""
    n1, e1 = geot_forward(sd, g1, num_layers)
    n2, e2 = geot_forward(sd, g2, num_layers)
    logits = head_forward(sd, pair_tensor(n1, n2), num_chunks)
    return logits, n1, e1, n2, e2
