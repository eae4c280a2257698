"""Residue graphs on the host side of the boundary.

``ResidueGraph`` is a minimal DGLGraph look-alike (``ndata``/``edata`` dicts, ``edges()``,
``nodes()``, ``num_nodes()``, ``batch_num_nodes()``, ``local_scope()``) so that code written
against the reference's DGLGraph usage in the hot path (deepinteract_modules.py:1426-1466,
1660-1679) runs unchanged; real ``dgl.DGLGraph`` objects are accepted too (duck typing).

``GraphBatch`` is the kernels' view of a batch of chains: concatenated, GLOBAL int32 ids,
destination-major CSR (csrc ``di_graph``).
"""
from __future__ import annotations

import contextlib
from typing import Sequence

import torch

from .config import NODE_COUNT_LIMIT
from ._lib import DI_GRAPH_GEO_REF, DiGraph

# edge_f[:, 20:27] of every edge as the reference featuriser produces them: direction (0, 0, 0),
# orientation quaternion (0, 0, 0, 1) (csrc di_graph.flags, DI_GRAPH_GEO_REF)
GEO_REF_COLS = (20, 27)
GEO_REF_VALUES = (0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0)


def edge_feats_geo_ref(edge_f: torch.Tensor) -> bool:
    """True when every edge's direction / orientation columns are the reference featuriser's
    constants (one device reduction and a host sync; the device builder knows it by construction)."""
    if edge_f is None or edge_f.dim() != 2 or edge_f.shape[0] == 0 or edge_f.shape[1] < GEO_REF_COLS[1]:
        return False
    ref = torch.tensor(GEO_REF_VALUES, dtype=edge_f.dtype, device=edge_f.device)
    return bool((edge_f[:, GEO_REF_COLS[0]:GEO_REF_COLS[1]] == ref).all())


class ResidueGraph:
    def __init__(self, src, dst, num_nodes: int, device=None):
        self._src = torch.as_tensor(src, device=device).long()
        self._dst = torch.as_tensor(dst, device=device).long()
        self._n = int(num_nodes)
        self.ndata: dict = {}
        self.edata: dict = {}
        self._bnn = torch.tensor([self._n])
        self._bne = torch.tensor([self._src.numel()])

    # --- DGLGraph-compatible surface used on the hot path
    def edges(self, form="uv"):
        return self._src, self._dst

    def nodes(self):
        return torch.arange(self._n, device=self._src.device)

    def num_nodes(self):
        return self._n

    number_of_nodes = num_nodes

    def num_edges(self):
        return int(self._src.numel())

    number_of_edges = num_edges

    def batch_num_nodes(self):
        return self._bnn

    def batch_num_edges(self):
        return self._bne

    def set_batch_num_nodes(self, v):
        self._bnn = v

    def set_batch_num_edges(self, v):
        self._bne = v

    @property
    def device(self):
        return self._src.device

    def to(self, device):
        g = ResidueGraph(self._src.to(device), self._dst.to(device), self._n)
        g.ndata = {k: v.to(device) for k, v in self.ndata.items()}
        g.edata = {k: v.to(device) for k, v in self.edata.items()}
        g._bnn, g._bne = self._bnn, self._bne
        return g

    @contextlib.contextmanager
    def local_scope(self):
        nd, ed = dict(self.ndata), dict(self.edata)
        try:
            yield
        finally:
            self.ndata.clear(); self.ndata.update(nd)
            self.edata.clear(); self.edata.update(ed)


def batch(graphs: Sequence[ResidueGraph]) -> ResidueGraph:
    """dgl.batch equivalent (ids offset, features concatenated, batch_num_* recorded)."""
    srcs, dsts, off = [], [], 0
    for g in graphs:
        s, d = g.edges()
        srcs.append(s + off)
        dsts.append(d + off)
        off += g.num_nodes()
    bg = ResidueGraph(torch.cat(srcs), torch.cat(dsts), off)
    for key in graphs[0].ndata:
        bg.ndata[key] = torch.cat([g.ndata[key] for g in graphs])
    for key in graphs[0].edata:
        bg.edata[key] = torch.cat([g.edata[key] for g in graphs])
    bg._bnn = torch.tensor([g.num_nodes() for g in graphs])
    bg._bne = torch.tensor([g.num_edges() for g in graphs])
    return bg


def unbatch(bg) -> list:
    out, noff, eoff = [], 0, 0
    src, dst = bg.edges()
    for n, e in zip(bg.batch_num_nodes().tolist(), bg.batch_num_edges().tolist()):
        g = ResidueGraph(src[eoff:eoff + e] - noff, dst[eoff:eoff + e] - noff, n)
        for key, val in bg.ndata.items():
            g.ndata[key] = val[noff:noff + n]
        for key, val in bg.edata.items():
            g.edata[key] = val[eoff:eoff + e]
        out.append(g)
        noff += n
        eoff += e
    return out


class GraphBatch:
    """Device-resident kernel view of a batch of chain graphs.

    Per-graph semantics are those of the reference at batch size 1 (the reference's
    batch>1 path indexes neighbour-edge ids locally and positional embeddings globally;
    SURVEY.md Appendix A.10): neighbour ids are offset into global edge ids and the
    positional-embedding row is the node's index within its own chain.
    """

    def __init__(self, src, dst, nbr, node_f, edge_f, nodes_per_graph, edges_per_graph,
                 node_count_limit=NODE_COUNT_LIMIT, in_ptr=None, node_pos=None, geo_ref=None,
                 _trusted_geo_ref=None):
        """in_ptr / node_pos: precomputed by the device builder (di_knn_graph); when given, the
        destination-major order is guaranteed by construction and not re-checked on the host.
        geo_ref: whether every edge carries the reference featuriser's constant direction /
        orientation columns (di_graph.flags DI_GRAPH_GEO_REF): None = check edge_f; True = claimed by
        the caller and verified (ValueError if the columns are not the constants: the kernels would
        skip a branch that is not zero); False = the general path.
        _trusted_geo_ref: package-internal (device builder, select_graphs, concat_batches), a value
        known by construction; not checked."""
        self.src, self.dst, self.nbr = src, dst, nbr
        self.node_f, self.edge_f = node_f, edge_f
        self.nodes_per_graph = [int(x) for x in nodes_per_graph]
        self.edges_per_graph = [int(x) for x in edges_per_graph]
        dev = src.device
        self.num_nodes = int(sum(self.nodes_per_graph))
        self.num_edges = int(sum(self.edges_per_graph))
        # max_num_graph_nodes of the model (LitGINI hyper-parameter, default NODE_COUNT_LIMIT = 2304):
        # the row count of InitEdge's positional nn.Embedding
        self.node_count_limit = int(node_count_limit)
        for n in self.nodes_per_graph:
            if n > self.node_count_limit:
                # the reference's nn.Embedding(max_num_graph_nodes) raises IndexError (:153, :210)
                raise IndexError(f"chain of {n} residues exceeds NODE_COUNT_LIMIT={self.node_count_limit}")
        if (in_ptr is None) != (node_pos is None):
            raise ValueError("in_ptr and node_pos come together")
        if in_ptr is not None:
            self.in_ptr, self.node_pos = in_ptr, node_pos
        else:
            self.node_pos = torch.cat([torch.arange(n, dtype=torch.int32, device=dev)
                                       for n in self.nodes_per_graph])
            if self.num_edges and bool((self.dst[1:] < self.dst[:-1]).any()):
                raise ValueError("edges must be destination-major (sorted by dst), as dgl.knn_graph emits them")
            counts = torch.bincount(self.dst.long(), minlength=self.num_nodes)
            self.in_ptr = torch.zeros(self.num_nodes + 1, dtype=torch.int32, device=dev)
            self.in_ptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
        self.node_off = [0]
        self.edge_off = [0]
        for n, e in zip(self.nodes_per_graph, self.edges_per_graph):
            self.node_off.append(self.node_off[-1] + n)
            self.edge_off.append(self.edge_off[-1] + e)
        if _trusted_geo_ref is not None:
            self.geo_ref = bool(_trusted_geo_ref) and self.num_edges > 0
        elif geo_ref is None:
            self.geo_ref = edge_feats_geo_ref(edge_f)
        elif geo_ref and self.num_edges == 0:
            self.geo_ref = False  # no edges: nothing to skip (as the trusted path does)
        elif geo_ref:
            if not edge_feats_geo_ref(edge_f):
                raise ValueError("geo_ref=True but the edge features do not carry the reference featuriser's "
                                 "constant direction / orientation columns (edge_f[:, 20:27])")
            self.geo_ref = True
        else:
            self.geo_ref = False
        self._c = DiGraph(self.num_nodes, self.num_edges, self.src.data_ptr(), self.dst.data_ptr(),
                          self.nbr.data_ptr(), self.node_pos.data_ptr(), self.in_ptr.data_ptr(),
                          DI_GRAPH_GEO_REF if self.geo_ref else 0)

    def with_geo_ref(self, on: bool) -> "GraphBatch":
        """The same batch with the DI_GRAPH_GEO_REF property set or cleared (clearing always keeps
        results exact; setting it is only valid when edge_feats_geo_ref(edge_f) holds)."""
        if on and not edge_feats_geo_ref(self.edge_f):
            raise ValueError("edge features do not carry the reference featuriser's constant direction / orientation")
        gb = GraphBatch.__new__(GraphBatch)
        gb.__dict__.update(self.__dict__)
        gb.geo_ref = bool(on)
        gb._c = DiGraph(self.num_nodes, self.num_edges, self.src.data_ptr(), self.dst.data_ptr(),
                        self.nbr.data_ptr(), self.node_pos.data_ptr(), self.in_ptr.data_ptr(),
                        DI_GRAPH_GEO_REF if on else 0)
        return gb

    @property
    def c_graph(self) -> DiGraph:
        return self._c

    @classmethod
    def from_graphs(cls, graphs, device=None, node_count_limit=NODE_COUNT_LIMIT):
        """From ResidueGraph / DGLGraph objects carrying ndata['f'] [N,113] (raw node features),
        edata['f'] [E,28], edata['src_nbr_e_ids'|'dst_nbr_e_ids'] [E,2] (per-graph local ids)."""
        srcs, dsts, nbrs, nfs, efs, nn, ne = [], [], [], [], [], [], []
        noff = eoff = 0
        for g in graphs:
            s, d = g.edges()
            dev = device or s.device
            srcs.append(s.to(dev).to(torch.int32) + noff)
            dsts.append(d.to(dev).to(torch.int32) + noff)
            nb = torch.cat([g.edata["src_nbr_e_ids"], g.edata["dst_nbr_e_ids"]], 1).to(dev)
            nbrs.append(nb.to(torch.int32) + eoff)
            nfs.append(g.ndata["f"].to(dev, torch.float32))
            efs.append(g.edata["f"].to(dev, torch.float32))
            nn.append(g.num_nodes())
            ne.append(g.num_edges())
            noff += g.num_nodes()
            eoff += g.num_edges()
        return cls(torch.cat(srcs).contiguous(), torch.cat(dsts).contiguous(), torch.cat(nbrs).contiguous(),
                   torch.cat(nfs).contiguous(), torch.cat(efs).contiguous(), nn, ne, node_count_limit=node_count_limit)

    @classmethod
    def from_arrays(cls, items, device, node_count_limit=NODE_COUNT_LIMIT):
        """items: dicts with num_nodes, src, dst, src_nbr, dst_nbr (local), node_f, edge_f."""
        srcs, dsts, nbrs, nfs, efs, nn, ne = [], [], [], [], [], [], []
        noff = eoff = 0
        for it in items:
            n, s = int(it["num_nodes"]), torch.as_tensor(it["src"])
            e = s.numel()
            srcs.append(s.to(torch.int32) + noff)
            dsts.append(torch.as_tensor(it["dst"]).to(torch.int32) + noff)
            nb = torch.cat([torch.as_tensor(it["src_nbr"]), torch.as_tensor(it["dst_nbr"])], 1)
            nbrs.append(nb.to(torch.int32) + eoff)
            nfs.append(torch.as_tensor(it["node_f"], dtype=torch.float32))
            efs.append(torch.as_tensor(it["edge_f"], dtype=torch.float32))
            nn.append(n)
            ne.append(e)
            noff += n
            eoff += e
        cat = lambda xs: torch.cat(xs).to(device).contiguous()  # noqa: E731
        return cls(cat(srcs), cat(dsts), cat(nbrs), cat(nfs), cat(efs), nn, ne, node_count_limit=node_count_limit)


def concat_batches(batches: Sequence[GraphBatch]) -> GraphBatch:
    """Device-side concatenation of GraphBatches (ids re-offset; new buffers; no host sync)."""
    srcs, dsts, nbrs, nfs, efs, ptrs, poss, nn, ne = [], [], [], [], [], [], [], [], []
    noff = eoff = 0
    for b in batches:
        srcs.append(b.src + noff)
        dsts.append(b.dst + noff)
        nbrs.append(b.nbr + eoff)
        nfs.append(b.node_f)
        efs.append(b.edge_f)
        ptrs.append(b.in_ptr[:-1] + eoff)
        poss.append(b.node_pos)
        nn += b.nodes_per_graph
        ne += b.edges_per_graph
        noff += b.num_nodes
        eoff += b.num_edges
    ptrs.append(torch.full((1,), eoff, dtype=torch.int32, device=batches[0].src.device))
    return GraphBatch(torch.cat(srcs).contiguous(), torch.cat(dsts).contiguous(), torch.cat(nbrs).contiguous(),
                      torch.cat(nfs).contiguous(), torch.cat(efs).contiguous(), nn, ne,
                      node_count_limit=max(b.node_count_limit for b in batches),
                      in_ptr=torch.cat(ptrs).contiguous(), node_pos=torch.cat(poss).contiguous(),
                      _trusted_geo_ref=all(b.geo_ref for b in batches))


def select_graphs(gb: GraphBatch, indices: Sequence[int]) -> GraphBatch:
    """A new GraphBatch of the chains ``indices`` of ``gb`` (in that order), ids re-offset."""
    parts = []
    for g in indices:
        n0, n1 = gb.node_off[g], gb.node_off[g + 1]
        e0, e1 = gb.edge_off[g], gb.edge_off[g + 1]
        parts.append(GraphBatch(gb.src[e0:e1] - n0, gb.dst[e0:e1] - n0, gb.nbr[e0:e1] - e0, gb.node_f[n0:n1],
                                gb.edge_f[e0:e1], [n1 - n0], [e1 - e0], node_count_limit=gb.node_count_limit,
                                in_ptr=gb.in_ptr[n0:n1 + 1] - e0, node_pos=gb.node_pos[n0:n1],
                                _trusted_geo_ref=gb.geo_ref))
    return concat_batches(parts)
