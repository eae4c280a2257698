"""On-device residue-graph builder (host sequencing of di_knn_topk / di_geo_feats /
di_build_nbr_ids). Replaces convert_df_to_dgl_graph's tensor work
(deepinteract_utils.py:386-555): Cα kNN (graph_utils.py:107-108), geometric features
(protein_feature_utils.py:322-377 + :494-530) and neighbour-edge ids (:534-553).

Input chains are dicts of backbone [N,4,3], amide_norm [N,3], dips [N,106] (see synth.py).
Neighbour-edge ids are drawn on the device from a counter-based RNG (seeded, reproducible);
the reference's torch.randperm stream cannot be reproduced on the GPU, so parity for the ids
is structural (tests/test_gpu_parity.py::test_nbr_ids_structure).
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


def knn(cas, k=KNN, device="cuda"):
    """cas: list of [N_g,3] Cα coordinate tensors -> (idx [Nt,k] int32 chain-local, d2 [Nt,k] f32)."""
    lib = _lib.load()
    sizes = [int(c.shape[0]) for c in cas]
    if min(sizes) < k:
        raise ValueError(f"a chain has fewer than k={k} residues")  # dgl.knn_graph raises too
    ca = torch.cat([torch.as_tensor(c, dtype=torch.float32) for c in cas]).to(device).contiguous()
    off = _node_off(sizes, device)
    nt = ca.shape[0]
    idx = torch.empty(nt, k, dtype=torch.int32, device=device)
    d2 = torch.empty(nt, k, dtype=torch.float32, device=device)
    _lib.check(lib.di_knn_topk(len(sizes), _p(off), _p(ca), k, max(sizes), _p(idx), _p(d2), _stream()),
               "di_knn_topk")
    return idx, d2


def build_graph_batch(chains, k=KNN, nb=GEO_NBRHD_SIZE, seed=0, device="cuda", return_aux=False,
                      node_count_limit=NODE_COUNT_LIMIT):
    """Build the kernels' GraphBatch for a list of chains entirely on the device."""
    if nb != 2:
        raise NotImplementedError("geo_nbrhd_size=2 (the reference's setting, lit_model_predict.py:156)")
    lib = _lib.load()
    sizes = [int(np.asarray(c["backbone"]).shape[0]) for c in chains]
    cat = lambda key, shape: torch.cat([torch.as_tensor(np.asarray(c[key]), dtype=torch.float32).reshape(shape)  # noqa: E731
                                        for c in chains]).to(device).contiguous()
    bb = cat("backbone", (-1, 4, 3))
    am = cat("amide_norm", (-1, 3))
    dips = cat("dips", (-1, 106))
    nt = bb.shape[0]
    idx, d2 = knn([bb[o:o + n, 1, :] for o, n in zip(np.cumsum([0] + sizes[:-1]), sizes)], k, device)
    off = _node_off(sizes, device)
    node_f = torch.empty(nt, 113, dtype=torch.float32, device=device)
    edge_f = torch.empty(nt * k, 28, dtype=torch.float32, device=device)
    stats = torch.empty(len(sizes), 4, dtype=torch.float32, device=device)
    args = _lib.DiGeoArgs(len(sizes), k, max(sizes), off.data_ptr(), bb.data_ptr(), am.data_ptr(), dips.data_ptr(),
                          idx.data_ptr(), d2.data_ptr(), node_f.data_ptr(), edge_f.data_ptr(), stats.data_ptr())
    _lib.check(lib.di_geo_feats(ctypes.byref(args), _stream()), "di_geo_feats")
    node_base = torch.repeat_interleave(off[:-1], torch.as_tensor(sizes, device=device))
    src = (idx + node_base[:, None]).reshape(-1).contiguous()
    dst = torch.arange(nt, dtype=torch.int32, device=device).repeat_interleave(k).contiguous()
    nbr = torch.empty(nt * k, 4, dtype=torch.int32, device=device)
    gb = GraphBatch(src, dst, nbr, node_f, edge_f, sizes, [n * k for n in sizes], node_count_limit=node_count_limit)
    _lib.check(lib.di_build_nbr_ids(gb.num_edges, _p(gb.src), _p(gb.dst), _p(gb.in_ptr), ctypes.c_uint64(seed),
                                    _p(nbr), _stream()), "di_build_nbr_ids")
    if return_aux:
        return gb, {"knn_idx": idx, "knn_d2": d2}
    return gb
