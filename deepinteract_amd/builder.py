"""On-device residue-graph builder (host sequencing of di_knn_topk / di_knn_graph /
di_geo_feats / di_build_nbr_ids[_torch]). Replaces convert_df_to_dgl_graph's tensor work
(deepinteract_utils.py:386-555): Cα kNN (graph_utils.py:107-108), geometric features
(protein_feature_utils.py:322-377 + :494-530) and neighbour-edge ids (:534-553).

Input chains are dicts of backbone [N,4,3], amide_norm [N,3], dips [N,106] (see synth.py).
One call builds every chain of a batch with one launch per stage (one host->device copy of the
inputs, no host synchronisation, no ATen glue between the kernels).

Neighbour-edge ids, two modes:
* ``nbr_seeds`` given (one int per chain): bit-exact with the reference — chain c's ids are the
  ones convert_df_to_dgl_graph draws right after ``torch.manual_seed(nbr_seeds[c])``
  (mt19937 + Fisher-Yates restated on the device, di_build_nbr_ids_torch);
* otherwise a counter-based RNG keyed by (seed, global edge id): same distribution, cheaper.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .config import GEO_NBRHD_SIZE, KNN, NODE_COUNT_LIMIT
from .graph import GraphBatch


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _node_off(sizes, device):
    off = np.zeros(len(sizes) + 1, dtype=np.int32)
    off[1:] = np.cumsum(sizes)
    return torch.as_tensor(off, device=device)


_stage = {"buf": None, "event": None}


BUILDER_MAX_NODES = 4096  # csrc/graph_builder.hip KNN_MAX_N: one chain's Cα rows staged in LDS


def _pinned(words):
    """Reusable pinned host staging buffer of at least `words` 4-byte words (float32 view)."""
    st = _stage
    if st["event"] is not None:
        st["event"].synchronize()  # the previous copy out of the buffer has finished
    if st["buf"] is None or st["buf"].numel() < words:
        st["buf"] = torch.empty(max(words, 1 << 20), dtype=torch.float32, pin_memory=True)
    return st["buf"]


def _keep_until_copied(buf):
    ev = torch.cuda.Event()
    ev.record()
    _stage["event"] = ev


def knn(cas, k=KNN, device="cuda"):
    """cas: list of [N_g,3] Cα coordinate tensors -> (idx [Nt,k] int32 chain-local, d2 [Nt,k] f32)."""
    sizes = [int(c.shape[0]) for c in cas]
    ca = torch.cat([torch.as_tensor(c, dtype=torch.float32) for c in cas]).to(device).contiguous()
    return _knn(ca, sizes, _node_off(sizes, device), k)


def _knn(ca, sizes, off, k):
    lib = _lib.load()
    if min(sizes) < k:
        raise ValueError(f"a chain has fewer than k={k} residues")  # dgl.knn_graph raises too
    nt = ca.shape[0]
    idx = torch.empty(nt, k, dtype=torch.int32, device=ca.device)
    d2 = torch.empty(nt, k, dtype=torch.float32, device=ca.device)
    _lib.check(lib.di_knn_topk(len(sizes), _p(off), _p(ca), k, max(sizes), _p(idx), _p(d2), _stream()),
               "di_knn_topk")
    return idx, d2


def build_graph_batch(chains, k=KNN, nb=GEO_NBRHD_SIZE, seed=0, device="cuda", return_aux=False,
                      node_count_limit=NODE_COUNT_LIMIT, nbr_seeds=None):
    """Build the kernels' GraphBatch for a list of chains entirely on the device.

    nbr_seeds: optional per-chain torch seeds (reference-exact neighbour ids, see module doc)."""
    if nb != 2:
        raise NotImplementedError("geo_nbrhd_size=2 (the reference's setting, lit_model_predict.py:156)")
    from .engine import gpu_device
    sizes = [int(np.asarray(c["backbone"]).shape[0]) for c in chains]
    for n in sizes:
        if n > node_count_limit:
            raise IndexError(f"chain of {n} residues exceeds NODE_COUNT_LIMIT={node_count_limit}")
        if n > BUILDER_MAX_NODES:
            raise NotImplementedError(f"chain of {n} residues: the on-device kNN handles chains of at most "
                                      f"{BUILDER_MAX_NODES} residues (di_knn_topk)")
    device = gpu_device(device)
    lib = _lib.load()
    if nbr_seeds is not None and len(nbr_seeds) != len(sizes):
        raise ValueError(f"{len(nbr_seeds)} neighbour seeds for {len(sizes)} chains")
    nt, G = int(sum(sizes)), len(sizes)
    # one host buffer -> one copy: [backbone nt x 12 | amide nt x 3 | dips nt x 106 | node offsets |
    # seeds], every field contiguous (memcpy-speed packing), staged in reusable pinned memory
    offs = np.zeros(G + 1, dtype=np.int64)
    offs[1:] = np.cumsum(sizes)
    n_off = (G + 2) // 2 * 2  # int32 offsets padded to 8 bytes, then the uint64 seeds
    n_meta = n_off + 2 * (len(nbr_seeds) if nbr_seeds is not None else 0)  # in 4-byte words
    m0 = (nt * 121 + 1) // 2 * 2  # metadata 8-byte aligned (uint64 seeds)
    words = m0 + n_meta
    stage = _pinned(words)
    hf = stage.numpy()
    np.concatenate([np.asarray(c["backbone"], dtype=np.float32).reshape(-1) for c in chains], out=hf[:nt * 12])
    np.concatenate([np.asarray(c["amide_norm"], dtype=np.float32).reshape(-1) for c in chains],
                   out=hf[nt * 12:nt * 15])
    np.concatenate([np.asarray(c["dips"], dtype=np.float32).reshape(-1) for c in chains], out=hf[nt * 15:nt * 121])
    hm = hf[m0:words].view(np.int32)
    hm[:n_off] = 0
    hm[:G + 1] = offs
    if nbr_seeds is not None:
        hm[n_off:].view(np.uint64)[:] = np.asarray(nbr_seeds, dtype=np.uint64)
    d_all = stage[:words].to(device, non_blocking=True)
    _keep_until_copied(stage)
    bb = d_all[:nt * 12].view(nt, 4, 3)
    am = d_all[nt * 12:nt * 15].view(nt, 3)
    dips = d_all[nt * 15:nt * 121].view(nt, 106)
    d_meta = d_all[m0:words].view(torch.int32)
    off = d_meta[:G + 1]
    ca = bb[:, 1, :].contiguous()
    idx, d2 = _knn(ca, sizes, off, k)
    node_f = torch.empty(nt, 113, dtype=torch.float32, device=device)
    edge_f = torch.empty(nt * k, 28, dtype=torch.float32, device=device)
    stats = torch.empty(G, 4, dtype=torch.float32, device=device)
    args = _lib.DiGeoArgs(G, k, max(sizes), off.data_ptr(), bb.data_ptr(), am.data_ptr(), dips.data_ptr(),
                          idx.data_ptr(), d2.data_ptr(), node_f.data_ptr(), edge_f.data_ptr(), stats.data_ptr())
    _lib.check(lib.di_geo_feats(ctypes.byref(args), _stream()), "di_geo_feats")
    src = torch.empty(nt * k, dtype=torch.int32, device=device)
    dst = torch.empty(nt * k, dtype=torch.int32, device=device)
    in_ptr = torch.empty(nt + 1, dtype=torch.int32, device=device)
    node_pos = torch.empty(nt, dtype=torch.int32, device=device)
    _lib.check(lib.di_knn_graph(G, _p(off), k, _p(idx), nt, _p(src), _p(dst), _p(in_ptr), _p(node_pos), _stream()),
               "di_knn_graph")
    nbr = torch.empty(nt * k, 4, dtype=torch.int32, device=device)
    if nbr_seeds is not None:
        seeds = d_meta[n_off:]
        _lib.check(lib.di_build_nbr_ids_torch(G, _p(off), k, _p(seeds), nt, _p(src), _p(dst), _p(nbr), _stream()),
                   "di_build_nbr_ids_torch")
    else:
        _lib.check(lib.di_build_nbr_ids(nt * k, _p(src), _p(dst), _p(in_ptr), ctypes.c_uint64(seed), _p(nbr),
                                        _stream()), "di_build_nbr_ids")
    # k_geo_feats writes the featuriser's constant direction / orientation columns (0,0,0,0,0,0,1)
    # for every edge, so the batch carries DI_GRAPH_GEO_REF by construction (no device check)
    gb = GraphBatch(src, dst, nbr, node_f, edge_f, sizes, [n * k for n in sizes], node_count_limit=node_count_limit,
                    in_ptr=in_ptr, node_pos=node_pos, _trusted_geo_ref=True)
    gb._keep = (d_all,)  # inputs referenced by in-flight launches
    if return_aux:
        return gb, {"knn_idx": idx, "knn_d2": d2}
    return gb
