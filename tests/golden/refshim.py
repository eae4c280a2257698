"""Fixture-generation shim: lets the reference's own Python modules run UNMODIFIED in this
container so that golden vectors come from the reference code itself.

TEST INFRASTRUCTURE ONLY. Used by ``tests/golden/make_golden.py`` in the build container,
never imported by the product (``deepinteract_amd``), never shipped to the GPU box as a
dependency of anything that runs there (``/root/reference`` does not exist there).

What is restated here
---------------------
DGL 0.6 (``environment.yml:28`` pins ``dgl-cu110==0.6``) is a third-party dependency that is
not vendored in the reference and not installed in this image. This module restates the
published semantics of exactly the DGL entry points the hot path calls:

* ``dgl.knn_graph(x, k)`` (bruteforce-blas, DGL 0.6 ``transform._knn_graph_blas``): pairwise
  squared distance by expansion ``x2 + x2^T - 2 x x^T``, per-row ascending top-k; edges are
  ``src = topk_idx[i, r]``, ``dst = i``, edge id ``i*k + r`` (called at graph_utils.py:107).
* ``dgl.nn.pytorch.pairwise_squared_distance`` (graph_utils.py:108).
* ``DGLGraph.apply_edges(udf)`` with an ``EdgeBatch`` exposing ``src``/``dst``/``data``
  (deepinteract_modules.py:78-91, :262, :453).
* ``DGLGraph.send_and_recv(eids, fn.u_mul_e | fn.copy_e, fn.sum)`` -> per-destination sums
  (deepinteract_modules.py:95-96).
* ``in_edges`` / ``edge_ids`` / ``local_scope`` / ``batch`` / ``unbatch`` /
  ``batch_num_nodes`` (deepinteract_utils.py:534-549, deepinteract_modules.py:1438-1463, 1677).

Every other missing import of the reference (pytorch_lightning, torchmetrics, wandb, atom3,
Bio, biopandas, parallel, timm, torchvision) is replaced by an inert stub: none of them
computes anything on the hot path (LightningModule is given the plain ``nn.Module``
behaviour the forward needs).
"""
from __future__ import annotations

import contextlib
import sys
import types

import torch
import torch.nn as nn

REFERENCE_ROOT = "/root/reference"


# ----------------------------------------------------------------------------------------
# Inert stubs for non-hot-path imports
# ----------------------------------------------------------------------------------------
class _Dummy:
    """Callable, subclassable, attribute-tolerant placeholder."""

    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Dummy()

    def __getattr__(self, name):
        return _Dummy()


class _StubModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        cls = type(name, (_Dummy,), {})
        setattr(self, name, cls)
        return cls


def _stub(name: str) -> types.ModuleType:
    if name in sys.modules:
        return sys.modules[name]
    mod = _StubModule(name)
    mod.__path__ = []  # behave as a package
    sys.modules[name] = mod
    parent, _, child = name.rpartition(".")
    if parent:
        setattr(_stub(parent), child, mod)
    return mod


class _LightningModule(nn.Module):
    """Only what LitGINI's forward path touches."""

    def save_hyperparameters(self, *a, **k):
        pass

    def log(self, *a, **k):
        pass

    @property
    def device(self):
        for p in self.parameters():
            return p.device
        return torch.device("cpu")


# ----------------------------------------------------------------------------------------
# DGL 0.6 restatement
# ----------------------------------------------------------------------------------------
class _LazyNodeView(dict):
    """edges.src / edges.dst: node fields gathered at the edge endpoints on access."""

    def __init__(self, ndata, idx):
        super().__init__()
        self._ndata, self._idx = ndata, idx

    def __getitem__(self, key):
        return self._ndata[key][self._idx]


class EdgeBatch:
    def __init__(self, g):
        self.src = _LazyNodeView(g.ndata, g._src)
        self.dst = _LazyNodeView(g.ndata, g._dst)
        self.data = g.edata


class DGLGraph:
    def __init__(self, src, dst, num_nodes=None):
        self._src = torch.as_tensor(src).long()
        self._dst = torch.as_tensor(dst).long()
        n = int(num_nodes) if num_nodes is not None else int(max(self._src.max(), self._dst.max()) + 1)
        self._n = n
        self.ndata = {}
        self.edata = {}
        self._bnn = torch.tensor([n])
        self._bne = torch.tensor([self._src.numel()])

    # --- structure ---
    def edges(self, form="uv"):
        return self._src, self._dst

    def nodes(self):
        return torch.arange(self._n)

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

    def in_edges(self, v):
        """For each vid in ``v`` (duplicates kept, in order) all (u, vid) in edge-id order."""
        v = torch.as_tensor(v).long().reshape(-1)
        order = torch.argsort(self._dst, stable=True)
        counts = torch.bincount(self._dst, minlength=self._n)
        ptr = torch.zeros(self._n + 1, dtype=torch.long)
        ptr[1:] = torch.cumsum(counts, 0)
        us, vs = [], []
        for vid in v.tolist():
            eids = order[ptr[vid]:ptr[vid + 1]]
            us.append(self._src[eids])
            vs.append(self._dst[eids])
        return torch.cat(us), torch.cat(vs)

    def edge_ids(self, u, v):
        key = {}
        for e, (a, b) in enumerate(zip(self._src.tolist(), self._dst.tolist())):
            key.setdefault((a, b), e)
        return torch.tensor([key[(a, b)] for a, b in zip(torch.as_tensor(u).tolist(),
                                                           torch.as_tensor(v).tolist())])

    # --- message passing ---
    @contextlib.contextmanager
    def local_scope(self):
        nd, ed = dict(self.ndata), dict(self.edata)
        try:
            yield
        finally:
            self.ndata.clear(); self.ndata.update(nd)
            self.edata.clear(); self.edata.update(ed)

    def apply_edges(self, func, edges="__ALL__"):
        out = func(EdgeBatch(self))
        for k, val in out.items():
            self.edata[k] = val

    def send_and_recv(self, edges, message_func, reduce_func):
        src, dst = edges
        src, dst = torch.as_tensor(src).long(), torch.as_tensor(dst).long()
        kind, a, b, out = message_func
        if kind == "u_mul_e":
            msg = self.ndata[a][src] * self.edata[b]
        elif kind == "copy_e":
            msg = self.edata[a]
        else:
            raise NotImplementedError(kind)
        rkind, rin, rout = reduce_func
        assert rkind == "sum" and rin == out
        acc = torch.zeros((self._n,) + tuple(msg.shape[1:]), dtype=msg.dtype)
        acc.index_add_(0, dst, msg)
        self.ndata[rout] = acc


def _pairwise_squared_distance(x):
    x2s = torch.sum(x * x, -1, keepdim=True)
    return x2s + x2s.transpose(-1, -2) - 2 * x @ x.transpose(-1, -2)


def _knn_graph(x, k):
    dist = _pairwise_squared_distance(x)
    k_idx = torch.topk(dist, k, dim=-1, largest=False)[1]
    n = x.shape[0]
    src = k_idx.reshape(-1)
    dst = torch.arange(n).repeat_interleave(k)
    return DGLGraph(src, dst, n)


def _batch(graphs):
    srcs, dsts, off = [], [], 0
    for g in graphs:
        srcs.append(g._src + off)
        dsts.append(g._dst + off)
        off += g._n
    bg = DGLGraph(torch.cat(srcs), torch.cat(dsts), off)
    for key in graphs[0].ndata:
        bg.ndata[key] = torch.cat([g.ndata[key] for g in graphs])
    for key in graphs[0].edata:
        bg.edata[key] = torch.cat([g.edata[key] for g in graphs])
    bg._bnn = torch.tensor([g._n for g in graphs])
    bg._bne = torch.tensor([g.num_edges() for g in graphs])
    return bg


def _unbatch(bg):
    out, noff, eoff = [], 0, 0
    for n, e in zip(bg._bnn.tolist(), bg._bne.tolist()):
        g = DGLGraph(bg._src[eoff:eoff + e] - noff, bg._dst[eoff:eoff + e] - noff, n)
        for key, val in bg.ndata.items():
            g.ndata[key] = val[noff:noff + n]
        for key, val in bg.edata.items():
            g.edata[key] = val[eoff:eoff + e]
        out.append(g)
        noff += n
        eoff += e
    return out


def _install_dgl():
    dgl = _stub("dgl")
    dgl.DGLGraph = DGLGraph
    dgl.graph = lambda uv, num_nodes=None, **k: DGLGraph(uv[0], uv[1], num_nodes)
    dgl.knn_graph = _knn_graph
    dgl.batch = _batch
    dgl.unbatch = _unbatch
    fn = _stub("dgl.function")
    fn.u_mul_e = lambda a, b, out: ("u_mul_e", a, b, out)
    fn.copy_e = lambda a, out: ("copy_e", a, None, out)
    fn.sum = lambda msg, out: ("sum", msg, out)
    udf = _stub("dgl.udf")
    udf.EdgeBatch = EdgeBatch
    nnpt = _stub("dgl.nn.pytorch")
    nnpt.pairwise_squared_distance = _pairwise_squared_distance
    _stub("dgl.data")


_INSTALLED = False


def install():
    """Install stubs + DGL restatement and put the reference on sys.path."""
    global _INSTALLED
    if _INSTALLED:
        return
    for name in ["wandb", "torchmetrics", "atom3", "atom3.case", "atom3.complex",
                 "atom3.conservation", "atom3.database", "atom3.neighbors", "atom3.pair",
                 "atom3.parse", "parallel", "Bio", "Bio.PDB", "Bio.PDB.PDBParser",
                 "Bio.PDB.Polypeptide", "Bio.PDB.DSSP", "Bio.PDB.ResidueDepth",
                 "Bio.PDB.vectors", "Bio.SCOP", "Bio.SCOP.Raf", "Bio.Align", "Bio.Seq",
                 "Bio.SeqRecord", "Bio.SeqIO", "biopandas", "biopandas.pdb", "timm",
                 "torchvision", "torchvision.models", "torchvision.models.resnet",
                 "pytorch_lightning.loggers"]:
        _stub(name)
    pl = _stub("pytorch_lightning")
    pl.LightningModule = _LightningModule
    _install_dgl()
    if REFERENCE_ROOT not in sys.path:
        sys.path.insert(0, REFERENCE_ROOT)
    _INSTALLED = True


def reference_modules():
    """Import and return (deepinteract_modules, deepinteract_utils) from the reference."""
    install()
    from project.utils import deepinteract_modules as dm  # noqa: E402
    from project.utils import deepinteract_utils as du  # noqa: E402
    return dm, du
