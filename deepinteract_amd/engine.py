"""GeoT forward on the HIP kernels (host sequencing of the C ABI).

Per batch of chains (one launch per stage covers every chain of the batch):

    di_node_embed                    h0, QKV(layer 0)
    di_init_edge                     F0 = InitEdge(G), Fn0 = nbr_linear_0(F0)
    for layer l < L-1:
        di_edge_layer(intermediate)  alpha_l, F_{l+1}, Fn_{l+1}
        di_node_layer(intermediate)  h_{l+1}, QKV(layer l+1)
    di_edge_layer(final)             alpha_{L-1}
    di_node_layer(final)             h_L

This mirrors DGLGeometricTransformer.forward (deepinteract_modules.py:1426-1466): the
returned edge features are the last INTERMEDIATE layer's (the final layer updates nodes only).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .config import GeoTConfig
from .graph import GraphBatch
from .packing import PackedGeoT

_TORCH_DT = {"f32": torch.float32, "bf16": torch.bfloat16}
_DI_DT = {"f32": _lib.DI_F32, "bf16": _lib.DI_BF16}


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def gpu_device(device) -> torch.device:
    """The ROCm device the HIP kernels run on; anything else (e.g. 'cpu') raises: the kernels
    dereference device pointers, so host tensors must never reach them (no CPU fallback)."""
    if not torch.cuda.is_available():
        raise RuntimeError("deepinteract_amd HIP kernels need a ROCm GPU (no CPU fallback)")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError(f"deepinteract_amd HIP kernels run on a ROCm GPU, not on {dev}")
    return torch.device("cuda", torch.cuda.current_device() if dev.index is None else dev.index)


def check_on(device: torch.device, what: str, *tensors):
    """Every tensor handed to a kernel must live on the kernel's device."""
    for t in tensors:
        if t is not None and t.device != device:
            raise ValueError(f"{what}: tensor on {t.device}, the kernels run on {device}")


class _Ticker:
    """Records (start, end) event pairs around consecutive launches on the current stream."""

    def __init__(self, events):
        self.events, self.name, self.start = events, None, None

    def __call__(self, name):
        if self.events is None:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        if self.name is not None:
            self.events.setdefault(self.name, []).append((self.start, ev))
        self.name, self.start = name, ev


class GeoTEngine:
    """Holds packed device weights; runs the GeoT forward for a GraphBatch."""

    def __init__(self, state_dict, dtype: str = "f32", cfg: GeoTConfig = GeoTConfig(), device="cuda"):
        if cfg.num_gnn_hidden_channels != 128 or cfg.num_gnn_attention_heads != 4:
            raise NotImplementedError("the GeoT kernels are specialised for 128 hidden channels, 4 heads")
        self.device = gpu_device(device)
        self.lib = _lib.load()
        self.dtype, self.cfg = dtype, cfg
        # fragment order of the edge-layer / InitEdge blobs this library build reads (ABI 5)
        layout = self.lib.di_blob_layout(2, _DI_DT[dtype])
        init_layout = self.lib.di_blob_layout(1, _DI_DT[dtype])
        if layout not in (16, 32) or layout != self.lib.di_blob_layout(3, _DI_DT[dtype]) or init_layout not in (16, 32):
            raise RuntimeError(f"unexpected blob layouts {layout} / {init_layout}")
        self.packed = PackedGeoT(state_dict, dtype, cfg, self.device, edge_layout=layout, init_layout=init_layout)
        self._check_blob_sizes()
        self._ws = {}
        self._ws_views = {}
        # node layer as two launches (di_node_aggregate + di_node_update; bit-identical to the fused
        # di_node_layer): the segment reduction (16 lanes per destination) at full occupancy instead
        # of inside the MFMA kernel's one-block-per-CU grid
        self.split_node = True
        # bf16: the attention aggregation folded into the edge layer's epilogue (di_edge_layer_attn +
        # di_node_update_folded; takes precedence over split_node for bf16)
        self.fold_attn = False
        # reference-featurised batches: node embedding as the first blocks of the InitEdge launch
        # (di_embed_init_edge, bf16 or fp32) instead of a separate launch (default, round 4: serial
        # 101 us for both vs 19 + 108 us with the resident InitEdge after the embedding)
        self.fuse_embed_init = True
        # with fuse_embed_init off: bf16 reference-featurised batches run InitEdge with its weights
        # resident in LDS (di_init_edge_resident: one 12-wave block per CU at 168 VGPRs), else the
        # staged di_init_edge. The resident block cannot share a SIMD with a pair-stream wave, so the
        # overlapped schedule needs it off (pipeline.OverlappedSchedule checks)
        self.resident_init = True

    def _check_blob_sizes(self):
        p, dt = self.packed, _DI_DT[self.dtype]
        L = p.num_layers
        blobs = [(0, p.embed)] + [(1, p.init)] + \
            [(3 if li == L - 1 else 2, p.edge[li]) for li in range(L)] + \
            [(5 if li == L - 1 else 4, p.node[li]) for li in range(L)]
        for kind, (mat, vec) in blobs:
            want_m = self.lib.di_blob_bytes(kind, dt, 0)
            want_v = self.lib.di_blob_bytes(kind, dt, 1)
            got_m = mat.numel() * mat.element_size()
            got_v = vec.numel() * vec.element_size()
            if want_m != got_m or want_v != got_v:
                raise RuntimeError(f"weight blob {kind} size mismatch: {got_m}/{got_v} vs {want_m}/{want_v}")

    def workspace(self, num_nodes: int, num_edges: int, slot: int = 0):
        """Per-slot activation buffers (two slots let a consumer of slot s's outputs, e.g. the
        pair-tensor kernel on another stream, run while the next batch computes in slot 1-s).

        Slots only grow: a batch no larger than the slot's capacity gets views of the same
        memory. Before a slot's buffers are replaced the device is drained, because a consumer
        on another stream may still be reading them and the caching allocator would otherwise
        hand that memory to the next launch."""
        key = (slot, num_nodes, num_edges)
        views = self._ws_views.get(key)
        if views is not None:
            return views
        cap = self._ws.get(slot)
        if cap is None or cap[0][0] < num_nodes or cap[0][1] < num_edges:
            self._ws_views = {}
            if cap is not None:
                torch.cuda.synchronize(self.device)
            cn = max(num_nodes, cap[0][0] if cap else 0)
            ce = max(num_edges, cap[0][1] if cap else 0)
            dt, dev, H = _TORCH_DT[self.dtype], self.device, self.cfg.num_gnn_hidden_channels
            self._ws[slot] = cap = ((cn, ce), {
                "h": [torch.empty(cn, H, dtype=dt, device=dev) for _ in range(2)],
                "qkv": [torch.empty(cn, 3 * H, dtype=dt, device=dev) for _ in range(2)],
                "f": [torch.empty(ce, H, dtype=dt, device=dev) for _ in range(2)],
                "fn": [torch.empty(ce, H, dtype=dt, device=dev) for _ in range(2)],
                "alpha": torch.empty(ce, 4, dtype=torch.float32, device=dev),
                "attn": torch.empty(cn, H, dtype=torch.float32, device=dev),
                "parts": torch.empty(max(self.lib.di_attn_parts_bytes(ce), 4) // 4, dtype=torch.float32, device=dev),
                "hT": torch.empty(H * cn, dtype=dt, device=dev),
            })
        b, H = cap[1], self.cfg.num_gnn_hidden_channels
        # views of the slot's buffers, cached per batch shape (the issue path builds no tensors)
        views = self._ws_views[key] = {
            "h": [t[:num_nodes] for t in b["h"]], "qkv": [t[:num_nodes] for t in b["qkv"]],
            "f": [t[:num_edges] for t in b["f"]], "fn": [t[:num_edges] for t in b["fn"]],
            "alpha": b["alpha"][:num_edges], "attn": b["attn"][:num_nodes], "parts": b["parts"],
            "hT": b["hT"][:H * num_nodes].view(H, num_nodes),
        }
        return views

    def forward(self, gb: GraphBatch, clone: bool = True, events=None, slot: int = 0, hT_out=None, signal=None):
        """-> (node feats [Nt,128], edge feats [Et,128]) in the engine dtype.

        events: optional dict kernel-name -> list; (start, end) torch.cuda.Event pairs are recorded
        around every launch on the launch stream (for per-kernel timing in bench.py).
        hT_out: optional [128, Nt] buffer for the transposed final node features (the pair tensor's
        input; default: the slot's own). Either way it is self.last_hT afterwards.
        signal: optional (pair-queue state tensor, job): this forward's first launch marks `job` ready
        at its start -- a previous forward's hT, complete by stream order (include/deepinteract_amd.h,
        pair-tensor queue: the signal_job argument)."""
        lib, p, dt = self.lib, self.packed, _DI_DT[self.dtype]
        check_on(self.device, "GeoTEngine.forward", gb.src, gb.dst, gb.nbr, gb.node_f, gb.edge_f,
                 gb.node_pos, gb.in_ptr, hT_out)
        if max(gb.nodes_per_graph) > p.pos_src.shape[0]:
            # InitEdge gathers positional rows node_pos < max_num_graph_nodes (nn.Embedding, :153, :210)
            raise IndexError(f"chain of {max(gb.nodes_per_graph)} residues exceeds this model's "
                             f"max_num_graph_nodes={p.pos_src.shape[0]}")
        ws = self.workspace(gb.num_nodes, gb.num_edges, slot)
        if hT_out is not None and (hT_out.shape != (self.cfg.num_gnn_hidden_channels, gb.num_nodes)
                                   or hT_out.dtype != _TORCH_DT[self.dtype] or not hT_out.is_contiguous()):
            raise ValueError("hT_out must be a contiguous [128, num_nodes] tensor of the engine dtype")
        hT = ws["hT"] if hT_out is None else hT_out
        g = ctypes.byref(gb.c_graph)
        st = _stream()
        h, qkv, f, fn, alpha = ws["h"], ws["qkv"], ws["f"], ws["fn"], ws["alpha"]
        # DI_GRAPH_GEO_REF batches: the conformation module's neighbour messages are exactly zero
        # (include/deepinteract_amd.h), so the gathered silu(nbr_linear(F)) rows are neither
        # written nor read
        if gb.geo_ref:
            fn = [None, None]
        sq, sjob = (_ptr(signal[0]), int(signal[1])) if signal is not None else (_ptr(None), -1)
        tick = _Ticker(events)
        if self.fuse_embed_init and gb.geo_ref:
            tick("init_edge")
            _lib.check(lib.di_embed_init_edge(g, dt, gb.node_f.shape[1], _ptr(gb.node_f), _ptr(p.embed[0]), _ptr(p.embed[1]),
                                              _ptr(h[0]), _ptr(qkv[0]), _ptr(gb.edge_f), _ptr(p.init[0]),
                                              _ptr(p.init[1]), _ptr(p.pos_src), _ptr(p.pos_dst), _ptr(f[0]), sq, sjob,
                                              st), "di_embed_init_edge")
        else:
            tick("node_embed")
            _lib.check(lib.di_node_embed(g, dt, gb.node_f.shape[1], _ptr(gb.node_f), _ptr(p.embed[0]),
                                         _ptr(p.embed[1]), _ptr(h[0]), _ptr(qkv[0]), sq, sjob, st), "di_node_embed")
            tick("init_edge")
            if self.dtype == "bf16" and gb.geo_ref and self.resident_init:
                # the path's InitEdge weights resident in LDS (one block per CU): faster alone than the
                # staged kernel
                _lib.check(lib.di_init_edge_resident(g, _ptr(gb.edge_f), _ptr(p.init[0]), _ptr(p.init[1]),
                                                     _ptr(p.pos_src), _ptr(p.pos_dst), _ptr(f[0]), st),
                           "di_init_edge_resident")
            else:
                _lib.check(lib.di_init_edge(g, dt, _ptr(gb.edge_f), _ptr(p.init[0]), _ptr(p.init[1]),
                                            _ptr(p.pos_src), _ptr(p.pos_dst), _ptr(f[0]), _ptr(fn[0]), st),
                           "di_init_edge")
        L = p.num_layers
        cur = 0
        fold = self.fold_attn and self.dtype == "bf16"
        for li in range(L):
            final = li == L - 1
            nxt = 1 - cur
            em, ev = p.edge[li]
            nm, nv = p.node[li]
            tick("edge_layer_final" if final else "edge_layer")
            if fold:
                # edge layer + the attention segment sums of its rows; node update adds split rows
                _lib.check(lib.di_edge_layer_attn(g, dt, int(final), _ptr(gb.edge_f), _ptr(f[cur]), _ptr(fn[cur]),
                                                  _ptr(qkv[cur]), _ptr(em), _ptr(ev), _ptr(None),
                                                  _ptr(None if final else f[nxt]), _ptr(None if final else fn[nxt]),
                                                  _ptr(ws["attn"]), _ptr(ws["parts"]), st), "di_edge_layer_attn")
                tick("node_layer_final" if final else "node_layer")
                _lib.check(lib.di_node_update_folded(g, dt, int(final), _ptr(ws["attn"]), _ptr(ws["parts"]),
                                                     _ptr(h[cur]), _ptr(nm), _ptr(nv), _ptr(h[nxt]),
                                                     _ptr(None if final else qkv[nxt]), _ptr(hT if final else None),
                                                     st), "di_node_update_folded")
                if not final:
                    f_out = nxt
                cur = nxt
                continue
            _lib.check(lib.di_edge_layer(g, dt, int(final), _ptr(gb.edge_f), _ptr(f[cur]), _ptr(fn[cur]),
                                         _ptr(qkv[cur]), _ptr(em), _ptr(ev), _ptr(alpha),
                                         _ptr(None if final else f[nxt]), _ptr(None if final else fn[nxt]),
                                         st), "di_edge_layer")
            if self.split_node:
                # CSR segment reduction of the attention messages, then O_node / FFN / next Q,K,V
                tick("node_aggr")
                _lib.check(lib.di_node_aggregate(g, dt, _ptr(alpha), _ptr(qkv[cur]), _ptr(ws["attn"]), st),
                           "di_node_aggregate")
                tick("node_layer_final" if final else "node_layer")
                _lib.check(lib.di_node_update(g, dt, int(final), _ptr(ws["attn"]), _ptr(h[cur]), _ptr(nm), _ptr(nv),
                                              _ptr(h[nxt]), _ptr(None if final else qkv[nxt]),
                                              _ptr(hT if final else None), st), "di_node_update")
            else:
                tick("node_layer_final" if final else "node_layer")
                _lib.check(lib.di_node_layer(g, dt, int(final), _ptr(alpha), _ptr(h[cur]), _ptr(qkv[cur]),
                                             _ptr(nm), _ptr(nv), _ptr(h[nxt]), _ptr(None if final else qkv[nxt]),
                                             _ptr(hT if final else None), st), "di_node_layer")
            if not final:
                f_out = nxt
            cur = nxt
        tick(None)
        node_out = h[cur]
        self.last_hT = hT  # [128, Nt] transposed final node features (pair-tensor input)
        edge_out = f[f_out] if L > 1 else f[0]
        if clone:
            return node_out.clone(), edge_out.clone()
        return node_out, edge_out


class PairTensorOp:
    """construct_interact_tensor (deepinteract_utils.py:158-172) for a batch of complexes.

    The launch (di_pair_launch) belongs to this op: kernel "auto" | "lines" | "rows" | "vector",
    resident blocks (0: one per CU), waves per row/line block (0: 4) and ``beside`` (the schedule
    beside a concurrent GeoT stream: a bounded store queue, non-temporal stores). Every choice
    writes the same bytes."""

    KERNELS = {"auto": _lib.DI_PAIR_AUTO, "rows": _lib.DI_PAIR_ROWS, "vector": _lib.DI_PAIR_VECTOR,
               "lines": _lib.DI_PAIR_LINES}

    def __init__(self, device="cuda", kernel: str = "auto", blocks: int = 0, waves_per_block: int = 0,
                 beside: bool = False):
        self.device = gpu_device(device)
        self.lib = _lib.load()
        if kernel not in self.KERNELS:
            raise ValueError(f"pair kernel {kernel!r}: one of {sorted(self.KERNELS)}")
        self.kernel = kernel
        self.launch = _lib.DiPairLaunch(self.KERNELS[kernel], int(blocks), int(waves_per_block), int(bool(beside)))
        self._desc_cache = {}

    def descs(self, h1_rows, h2_rows, l1s, l2s, hidden):
        key = (tuple(h1_rows), tuple(h2_rows), tuple(l1s), tuple(l2s), hidden)
        if key not in self._desc_cache:
            arr = (_lib.DiPairDesc * len(l1s))()
            off = 0
            offs = []
            for i, (a, b, l1, l2) in enumerate(zip(h1_rows, h2_rows, l1s, l2s)):
                arr[i] = _lib.DiPairDesc(a, b, off, l1, l2)
                offs.append(off)
                off += 2 * hidden * l1 * l2
            t = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.device)
            self._desc_cache[key] = (t, offs, off)
        return self._desc_cache[key]

    def __call__(self, h, h1_rows, h2_rows, l1s, l2s, out=None, events=None, hT=None):
        """h: [rows, H] node features (both chains of every complex). Returns a flat buffer and
        the per-complex [1, 2H, L1, L2] views."""
        hidden = h.shape[1]
        dt = _lib.DI_BF16 if h.dtype == torch.bfloat16 else _lib.DI_F32
        if h.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError(h.dtype)
        check_on(self.device, "PairTensorOp", h, hT, out)
        d, offs, total = self.descs(h1_rows, h2_rows, l1s, l2s, hidden)
        if out is None:
            out = torch.empty(total, dtype=h.dtype, device=h.device)
        elif out.numel() < total:
            raise ValueError("pair-tensor output buffer too small")
        esz = h.element_size()
        vec = 16 // esz
        if hT is not None and (hT.shape != (hidden, h.shape[0]) or hT.dtype != h.dtype):
            raise ValueError("hT must be h transposed")
        aligned = int(hT is not None and h.shape[0] % vec == 0 and out.data_ptr() % 16 == 0
                      and all(l2 % vec == 0 for l2 in l2s) and all(o % vec == 0 for o in offs)
                      and all(r % vec == 0 for r in h2_rows))
        if aligned and out.data_ptr() % 128 == 0 and all(o * esz % 128 == 0 for o in offs) \
                and all(l1 * l2 * esz % 128 == 0 for l1, l2 in zip(l1s, l2s)):
            aligned = 2  # every channel plane starts on a 128-B line: whole-line stores
        need = {"lines": 2, "rows": 1, "vector": 1}.get(self.kernel, 0)
        if aligned < need:
            raise ValueError(f"pair kernel {self.kernel!r} needs {'128-B' if need == 2 else '16-B'} aligned planes "
                             f"and hT; this batch allows {['the generic', 'the 16-B', 'the 128-B'][aligned]} path")
        tick = _Ticker(events)
        tick("pair_tensor")
        _lib.check(self.lib.di_pair_tensor(dt, _ptr(d), len(l1s), max(l1s), max(l2s), hidden, aligned,
                                           _ptr(h.contiguous()), _ptr(hT), h.shape[0], ctypes.byref(self.launch),
                                           _ptr(out), _stream()), "di_pair_tensor")
        tick(None)
        views = [out[o:o + 2 * hidden * l1 * l2].view(1, 2 * hidden, l1, l2)
                 for o, l1, l2 in zip(offs, l1s, l2s)]
        return out, views


class HeadPrologueOp:
    """ELU(InstanceNorm2d(conv2d_1(T))) of the contact head for a batch of complexes, with the
    pair tensor T never materialised (di_head_prologue): the 1x1 conv of the
    outer concat separates per chain and the InstanceNorm statistics are analytic. Output: the
    head body's input, [1, C, L1, L2] per complex, in the dtype of h."""

    def __init__(self, conv_w, conv_b, in_gamma, in_beta, eps=1e-6, device="cuda"):
        self.device = gpu_device(device)
        self.lib = _lib.load()
        f = lambda t: t.detach().to(self.device, torch.float32).contiguous()  # noqa: E731
        self.w = f(conv_w).reshape(conv_w.shape[0], -1)  # [C, 2H(,1,1)] -> [C, 2H]
        self.b, self.g, self.beta = f(conv_b), f(in_gamma), f(in_beta)
        self.eps = float(eps)
        self.channels = self.w.shape[0]
        self._desc_cache = {}

    @classmethod
    def from_head(cls, head, device="cuda"):
        """From a ResNet2DInputWithOptAttention (conv2d_1 + inorm_1)."""
        return cls(head.conv2d_1.weight, head.conv2d_1.bias, head.inorm_1.weight, head.inorm_1.bias,
                   head.inorm_1.eps, device)

    def __call__(self, h, h1_rows, h2_rows, l1s, l2s, out=None, events=None):
        hidden, C = h.shape[1], self.channels
        if h.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError(h.dtype)
        check_on(self.device, "HeadPrologueOp", h, out)
        if self.w.shape[1] != 2 * hidden:
            raise ValueError(f"conv2d_1 expects {self.w.shape[1]} input channels, h gives 2x{hidden}")
        dt = _lib.DI_BF16 if h.dtype == torch.bfloat16 else _lib.DI_F32
        # descriptors with out_off in units of the [C, L1, L2] output
        key = ("prologue", tuple(h1_rows), tuple(h2_rows), tuple(l1s), tuple(l2s), C)
        if key not in self._desc_cache:
            arr = (_lib.DiPairDesc * len(l1s))()
            off, offs = 0, []
            for i, (a, b, l1, l2) in enumerate(zip(h1_rows, h2_rows, l1s, l2s)):
                arr[i] = _lib.DiPairDesc(a, b, off, l1, l2)
                offs.append(off)
                off += C * l1 * l2
            t = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.device)
            self._desc_cache[key] = (t, offs, off)
        d, offs, total = self._desc_cache[key]
        if out is None:
            out = torch.empty(total, dtype=h.dtype, device=h.device)
        elif out.numel() < total or out.dtype != h.dtype:
            raise ValueError("head-prologue output buffer too small or of the wrong dtype")
        m1, m2 = max(l1s), max(l2s)
        nbytes = self.lib.di_head_prologue_work_bytes(len(l1s), m1, m2, C)
        work = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=h.device)
        vec = 16 // h.element_size()
        aligned = out.data_ptr() % 16 == 0 and all(l2 % vec == 0 for l2 in l2s) and all(o % vec == 0 for o in offs)
        tick = _Ticker(events)
        tick("head_prologue")
        _lib.check(self.lib.di_head_prologue(dt, _ptr(d), len(l1s), m1, m2, hidden, C, int(aligned),
                                             _ptr(h.contiguous()), _ptr(self.w), _ptr(self.b), _ptr(self.g),
                                             _ptr(self.beta), self.eps, _ptr(work), _ptr(out), _stream()),
                   "di_head_prologue")
        tick(None)
        views = [out[o:o + C * l1 * l2].view(1, C, l1, l2) for o, l1, l2 in zip(offs, l1s, l2s)]
        return out, views

