"""Module-at-a-time drop-ins for the reference's GeoT building blocks.

Same constructor arguments, state-dict keys, forward signatures and results as
(/root/reference/project/utils/deepinteract_modules.py):

* ``InitEdgeModule.forward(graph) -> [E,128]``                                     (:128-264)
* ``ConformationModule.forward(graph, orig_edge_feats) -> [E,128]``                (:267-455)
* ``MultiHeadGeometricAttentionLayer.forward(graph, node, edge) -> (h [N,4,32], e_out [E,4,32] | None)``
                                                                                   (:34-121)
* ``GeometricTransformerModule.forward(graph, orig_edge_feats) -> (node, edge)``   (:500-733)
* ``FinalGeometricTransformerModule.forward(graph, orig_edge_feats) -> node``      (:735-952)

Each module loads its OWN reference state dict (``load_reference_state_dict``; keys as the
reference module's ``state_dict()``), folds BatchNorm on the host and runs on the HIP kernels:
di_init_edge / di_conformation (the fused edge kernel stopped after the conformation output),
di_gemm_bias_act for every Linear and di_geo_attention for propagate_attention. The fused
whole-transformer path (modules.DGLGeometricTransformer / engine.GeoTEngine) is the fast path;
these exist so code that calls the reference modules one at a time finds them. Eval mode only
(dropout is the identity, BatchNorm uses running statistics), like the reference's predict path.
Graphs: ResidueGraph or DGLGraph (batched graphs get per-chain semantics, as everywhere here).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .config import GeoTConfig
from .graph import GraphBatch, ResidueGraph, unbatch
from .packing import (bn_affine, edge_blob, fold_bn_before, init_blob, lin, pack_matrix_natural)

_DI_DT = {"f32": _lib.DI_F32, "bf16": _lib.DI_BF16}
_TORCH_DT = {"f32": torch.float32, "bf16": torch.bfloat16}


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _graphs(graph):
    if hasattr(graph, "batch_num_nodes") and len(graph.batch_num_nodes()) > 1:
        return unbatch(graph) if isinstance(graph, ResidueGraph) else __import__("dgl").unbatch(graph)
    return [graph]


def _topology(graph, device):
    """Kernel view (global ids, CSR) of a (batched) graph; features are passed separately."""
    gs = _graphs(graph)
    srcs, dsts, nbrs, nn_, ne = [], [], [], [], []
    noff = eoff = 0
    for g in gs:
        s, d = g.edges()
        srcs.append(s.to(device, torch.int32) + noff)
        dsts.append(d.to(device, torch.int32) + noff)
        if "src_nbr_e_ids" in g.edata:
            nb = torch.cat([g.edata["src_nbr_e_ids"], g.edata["dst_nbr_e_ids"]], 1).to(device, torch.int32) + eoff
        else:
            nb = torch.zeros(g.num_edges(), 4, dtype=torch.int32, device=device)
        nbrs.append(nb)
        nn_.append(g.num_nodes())
        ne.append(g.num_edges())
        noff += g.num_nodes()
        eoff += g.num_edges()
    empty = torch.empty(0, device=device)
    return GraphBatch(torch.cat(srcs).contiguous(), torch.cat(dsts).contiguous(), torch.cat(nbrs).contiguous(),
                      empty, empty, nn_, ne)


class _Base(nn.Module):
    def __init__(self, dtype="f32", device="cuda"):
        super().__init__()
        if not torch.cuda.is_available():
            raise RuntimeError("deepinteract_amd kernels need a ROCm GPU (no CPU fallback)")
        assert dtype in _DI_DT
        self.dtype = dtype
        self.device = torch.device(device)
        self.lib = _lib.load()
        self._w = {}

    def _t(self, x):
        return x.to(self.device, _TORCH_DT[self.dtype]).contiguous()

    def _dev_lin(self, name, w, b=None):
        """Register a packed Linear (numpy fp64 W [out,in], b [out] | None)."""
        bias = None if b is None else torch.as_tensor(np.asarray(b), dtype=torch.float32).to(self.device)
        self._w[name] = (pack_matrix_natural(w, self.dtype).to(self.device), bias, w.shape[0], w.shape[1])

    def _gemm(self, name, x, act=0, res=None):
        wp, bias, nout, nin = self._w[name]
        x = self._t(x)
        assert x.shape[1] == nin, (name, x.shape, nin)
        y = torch.empty(x.shape[0], nout, dtype=x.dtype, device=self.device)
        if res is not None:
            res = self._t(res)
        _lib.check(self.lib.di_gemm_bias_act(_DI_DT[self.dtype], x.shape[0], nin, nout, _ptr(x), x.stride(0),
                                             _ptr(wp), _ptr(bias), act, _ptr(res), 0 if res is None else res.stride(0),
                                             _ptr(y), y.stride(0), _stream()), f"di_gemm_bias_act({name})")
        return y

    def _out(self, t):
        return t.to(torch.float32) if self.dtype == "f32" else t


class InitEdgeModule(_Base):
    """deepinteract_modules.InitEdgeModule (:128-264): edge_f [E,28] -> [E,128]."""

    def load_reference_state_dict(self, sd):
        full = {f"M.{k}": v for k, v in sd.items()}
        # the fragment order this library build reads for the init blob (kind 1)
        layout = self.lib.di_blob_layout(1, _DI_DT[self.dtype])
        mat, vec, ps, pd = init_blob(full, self.dtype, p="M", nbr=None, layout=layout)
        self.blob = tuple(t.to(self.device).contiguous() for t in (mat, vec, ps, pd))
        return self

    def forward(self, graph):
        gb = _topology(graph, self.device)
        edge_f = torch.cat([g.edata["f"] for g in _graphs(graph)]).to(self.device, torch.float32).contiguous()
        f = torch.empty(gb.num_edges, 128, dtype=_TORCH_DT[self.dtype], device=self.device)
        fn = torch.empty_like(f)
        mat, vec, ps, pd = self.blob
        _lib.check(self.lib.di_init_edge(ctypes.byref(gb.c_graph), _DI_DT[self.dtype], _ptr(edge_f), _ptr(mat),
                                         _ptr(vec), _ptr(ps), _ptr(pd), _ptr(f), _ptr(fn), _stream()),
                   "di_init_edge")
        return self._out(f)


class ConformationModule(_Base):
    """deepinteract_modules.ConformationModule (:267-455). forward reads graph.edata['f'] (the
    current edge features, like the reference) and the neighbour-edge ids."""

    def load_reference_state_dict(self, sd):
        full = {f"M.{k}": v for k, v in sd.items()}
        mat, vec = edge_blob(full, 0, True, self.dtype, GeoTConfig(), conf_only=True, c="M")
        self.blob = (mat.to(self.device).contiguous(), vec.to(self.device).contiguous())
        self._dev_lin("nbr", *lin(full, "M.nbr_linear"))
        return self

    def run(self, gb, edge_feats, orig_edge_feats):
        F = self._t(edge_feats)
        fn = self._gemm("nbr", F, act=1)                        # silu(nbr_linear(F)), once per edge
        G = orig_edge_feats.to(self.device, torch.float32).contiguous()
        out = torch.empty_like(F)
        _lib.check(self.lib.di_conformation(ctypes.byref(gb.c_graph), _DI_DT[self.dtype], _ptr(G), _ptr(F), _ptr(fn),
                                            _ptr(self.blob[0]), _ptr(self.blob[1]), _ptr(out), _stream()),
                   "di_conformation")
        return out

    def forward(self, graph, orig_edge_feats):
        gb = _topology(graph, self.device)
        F = torch.cat([g.edata["f"] for g in _graphs(graph)])
        return self._out(self.run(gb, F, orig_edge_feats))


class MultiHeadGeometricAttentionLayer(_Base):
    """deepinteract_modules.MultiHeadGeometricAttentionLayer (:34-121)."""

    def __init__(self, num_input_feats=128, num_output_feats=32, num_heads=4, using_bias=False,
                 update_edge_feats=True, dtype="f32", device="cuda"):
        super().__init__(dtype, device)
        if num_input_feats != 128 or num_output_feats != 32 or num_heads != 4:
            raise NotImplementedError("kernels are specialised for 128 features = 4 heads x 32")
        self.using_bias, self.update_edge_feats = using_bias, update_edge_feats
        self.num_heads, self.num_output_feats = num_heads, num_output_feats

    def load_reference_state_dict(self, sd, node_bn=None, edge_bn=None):
        """node_bn / edge_bn: optional (scale, shift) of a BatchNorm applied to the inputs first
        (folded into Q/K/V and edge_feats_projection; used by the transformer modules)."""
        ws = [lin(sd, q) for q in ("Q", "K", "V")]
        if node_bn is not None:
            ws = [fold_bn_before(w, b, *node_bn) for w, b in ws]
        wq = np.concatenate([w for w, _ in ws])
        bq = np.concatenate([b for _, b in ws])
        self._dev_lin("qkv", wq, bq if (self.using_bias or node_bn is not None) else None)
        w, b = lin(sd, "edge_feats_projection")
        if edge_bn is not None:
            w, b = fold_bn_before(w, b, *edge_bn)
        self._dev_lin("proj", w, b if (self.using_bias or edge_bn is not None) else None)
        return self

    def run(self, gb, node_feats, edge_feats, want_e_out):
        qkv = self._gemm("qkv", node_feats)
        proj = self._gemm("proj", edge_feats)
        e_out = torch.empty_like(proj) if want_e_out else None
        alpha = torch.empty(gb.num_edges, 4, dtype=torch.float32, device=self.device)
        h = torch.empty(gb.num_nodes, 128, dtype=qkv.dtype, device=self.device)
        _lib.check(self.lib.di_geo_attention(ctypes.byref(gb.c_graph), _DI_DT[self.dtype], _ptr(qkv), _ptr(proj),
                                             _ptr(e_out), _ptr(alpha), _ptr(h), _stream()), "di_geo_attention")
        return h, e_out

    def forward(self, graph, node_feats, edge_feats):
        gb = _topology(graph, self.device)
        h, e_out = self.run(gb, node_feats, edge_feats, self.update_edge_feats)
        h = self._out(h).view(-1, self.num_heads, self.num_output_feats)
        if e_out is not None:
            e_out = self._out(e_out).view(-1, self.num_heads, self.num_output_feats)
        return h, e_out


class GeometricTransformerModule(_Base):
    """deepinteract_modules.GeometricTransformerModule (:500-733): one intermediate layer.
    forward(graph, orig_edge_feats) reads graph.ndata['f'] / graph.edata['f'] -> (node, edge)."""

    final = False

    def __init__(self, dtype="f32", device="cuda", **kwargs):
        super().__init__(dtype, device)
        self.conformation_module = ConformationModule(dtype, device)
        self.mha_module = MultiHeadGeometricAttentionLayer(update_edge_feats=not self.final, dtype=dtype,
                                                           device=device)

    def load_reference_state_dict(self, sd):
        sub = lambda pre: {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}  # noqa: E731
        self.conformation_module.load_reference_state_dict(sub("conformation_module."))
        self.mha_module.load_reference_state_dict(sub("mha_module."), node_bn=bn_affine(sd, "batch_norm1_node_feats"),
                                                  edge_bn=bn_affine(sd, "batch_norm1_edge_feats"))
        sides = ("node",) if self.final else ("node", "edge")
        for side in sides:
            self._dev_lin(f"O_{side}", *lin(sd, f"O_{side}_feats"))
            w1, b1 = fold_bn_before(*lin(sd, f"{side}_feats_MLP.0"), *bn_affine(sd, f"batch_norm2_{side}_feats"))
            self._dev_lin(f"{side}_mlp0", w1, b1)
            self._dev_lin(f"{side}_mlp3", *lin(sd, f"{side}_feats_MLP.3"))
        return self

    def _ffn(self, side, x_in1, attn_out):
        x = self._gemm(f"O_{side}", attn_out, res=x_in1)         # in1 + O(attn)
        t = self._gemm(f"{side}_mlp0", x, act=1)                 # SiLU(W1 BN2(x))
        return self._gemm(f"{side}_mlp3", t, res=x)              # x + W2 t

    def run(self, gb, node_feats, edge_feats, orig_edge_feats):
        n1, e1 = self._t(node_feats), self._t(edge_feats)
        conf = self.conformation_module.run(gb, e1, orig_edge_feats)
        h, e_out = self.mha_module.run(gb, n1, conf, not self.final)
        node = self._ffn("node", n1, h)
        edge = None if self.final else self._ffn("edge", e1, e_out)
        return node, edge

    def forward(self, graph, orig_edge_feats):
        gb = _topology(graph, self.device)
        gs = _graphs(graph)
        node, edge = self.run(gb, torch.cat([g.ndata["f"] for g in gs]), torch.cat([g.edata["f"] for g in gs]),
                              orig_edge_feats)
        return self._out(node), self._out(edge)


class FinalGeometricTransformerModule(GeometricTransformerModule):
    """deepinteract_modules.FinalGeometricTransformerModule (:735-952): nodes only."""

    final = True

    def forward(self, graph, orig_edge_feats):
        gb = _topology(graph, self.device)
        gs = _graphs(graph)
        node, _ = self.run(gb, torch.cat([g.ndata["f"] for g in gs]), torch.cat([g.edata["f"] for g in gs]),
                           orig_edge_feats)
        return self._out(node)


__all__ = ["InitEdgeModule", "ConformationModule", "MultiHeadGeometricAttentionLayer",
           "GeometricTransformerModule", "FinalGeometricTransformerModule"]
