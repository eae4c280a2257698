"""Reference-interface modules over the HIP kernels.

Mirrors the Python API the reference's hot path exposes (deepinteract_modules.py):

* ``DGLGeometricTransformer.forward(graph) -> graph`` (:1426-1466): reads ndata['f'] [N,128],
  edata['f'] [E,28], edata['src_nbr_e_ids'|'dst_nbr_e_ids'] [E,2]; writes ndata['f'] [N,128]
  and edata['f'] [E,128] (the last intermediate layer's edges) in place, keeps batch_num_*.
* ``LitGINI`` (:1478): ``gnn_forward`` (:1660-1679), ``shared_step`` (:1687-1745),
  ``predict_step`` (:2178-2184), plus ``predict_batch`` (the batched entry the benchmark and the
  distributed driver use).

Graphs may be ``deepinteract_amd.graph.ResidueGraph`` or real ``dgl.DGLGraph`` objects.
Batched graphs get per-chain semantics (each chain as the reference computes it at batch size 1).
Weights come from a reference-keyed state dict (``load_reference_state_dict``); the GeoT part
is packed once into device blobs, the head is a regular torch module.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .config import GeoTConfig, NODE_COUNT_LIMIT, RESIDUE_COUNT_LIMIT
from .engine import GeoTEngine, HeadPrologueOp, PairTensorOp, gpu_device
from .graph import GraphBatch, ResidueGraph, batch as batch_graphs, unbatch
from .head import HeadNormOps, ResNet2DInputWithOptAttention, contact_probs


def _identity_embedding_sd(sd, cfg: GeoTConfig):
    """Standalone DGLGeometricTransformer: node features arrive already embedded (128-d);
    reuse the fused embed kernel with an identity node_in_embedding."""
    out = {k: v for k, v in sd.items()}
    out["node_in_embedding.weight"] = torch.eye(cfg.num_gnn_hidden_channels)
    return out


def _graph_list(graph):
    if hasattr(graph, "batch_num_nodes") and len(graph.batch_num_nodes()) > 1:
        return unbatch(graph) if isinstance(graph, ResidueGraph) else __import__("dgl").unbatch(graph)
    return [graph]


class DGLGeometricTransformer(nn.Module):
    """Drop-in for deepinteract_modules.DGLGeometricTransformer (eval-mode forward)."""

    def __init__(self, node_count_limit=NODE_COUNT_LIMIT, num_hidden_channels=128, num_attention_heads=4,
                 knn=20, num_layers=4, dtype="f32", **kwargs):
        super().__init__()
        self.cfg = GeoTConfig(num_gnn_layers=num_layers, num_gnn_hidden_channels=num_hidden_channels,
                              num_gnn_attention_heads=num_attention_heads, knn=knn,
                              node_count_limit=node_count_limit, num_node_input_feats=num_hidden_channels)
        if num_hidden_channels != 128 or num_attention_heads != 4:
            raise NotImplementedError("kernels are specialised for 128 hidden channels, 4 heads")
        if node_count_limit <= 0:
            raise ValueError("max_num_graph_nodes must be positive")
        self.dtype = dtype
        self.engine = None

    def load_reference_state_dict(self, sd, prefix="gnn_module.0."):
        """Keys as in LitGINI's state dict; prefix strips to this module's own keys."""
        full = {("gnn_module.0." + k[len(prefix):]) if k.startswith(prefix) else k: v for k, v in sd.items()}
        self.engine = GeoTEngine(_identity_embedding_sd(full, self.cfg), self.dtype, self.cfg)
        return self

    def forward(self, graph):
        if self.engine is None:
            raise RuntimeError("load_reference_state_dict() first")
        bnn, bne = graph.batch_num_nodes(), graph.batch_num_edges()
        gb = GraphBatch.from_graphs(_graph_list(graph), device=self.engine.device,
                                     node_count_limit=self.cfg.node_count_limit)
        h, e = self.engine.forward(gb)
        graph.ndata["f"] = h.to(torch.float32) if self.dtype == "f32" else h
        graph.edata["f"] = e.to(torch.float32) if self.dtype == "f32" else e
        graph.set_batch_num_nodes(bnn)
        graph.set_batch_num_edges(bne)
        return graph


class LitGINI(nn.Module):
    """Inference-side drop-in for LitGINI (GeoT on HIP kernels, dilated-ResNet head on torch)."""

    def __init__(self, num_node_input_feats=113, num_gnn_layers=2, num_gnn_hidden_channels=128,
                 num_gnn_attention_heads=4, knn=20, num_interact_layers=14, num_interact_hidden_channels=128,
                 num_classes=2, max_num_graph_nodes=NODE_COUNT_LIMIT, max_num_residues=RESIDUE_COUNT_LIMIT,
                 dtype="f32", head_dtype=torch.float32, precise_head=False, fuse_head_prologue=False,
                 head_channels_last=False, head_hip_ops=True, **kwargs):
        super().__init__()
        if num_gnn_hidden_channels != 128 or num_gnn_attention_heads != 4:
            # Q/K/V are Linear(H, H) whatever the head count, so a checkpoint trained with another
            # head count would load and silently compute 4-head attention
            raise NotImplementedError("the GeoT kernels are specialised for 128 hidden channels, 4 heads")
        if max_num_graph_nodes <= 0:
            # the GeoT kernels need only node_pos < max_num_graph_nodes (the positional table's rows);
            # the on-device graph builder's own chain limit (4096) is enforced where it is used
            raise ValueError("max_num_graph_nodes must be positive")
        self.cfg = GeoTConfig(num_node_input_feats=num_node_input_feats, num_gnn_layers=num_gnn_layers,
                              num_gnn_hidden_channels=num_gnn_hidden_channels,
                              num_gnn_attention_heads=num_gnn_attention_heads, knn=knn,
                              node_count_limit=max_num_graph_nodes,
                              num_interact_layers=num_interact_layers,
                              num_interact_hidden_channels=num_interact_hidden_channels, num_classes=num_classes)
        self.dtype = dtype
        self.head_dtype = head_dtype
        # precise_head: run the head's convolutions without MIOpen's fast algorithms (Winograd /
        # FFT variants drift ~1e-3 relative over the 58 residual blocks); GEMM-based fp32 convs
        # keep logits within 1e-4 of the reference CPU path.
        self.precise_head = precise_head
        # fuse_head_prologue: ELU(inorm_1(conv2d_1(T))) straight from the node features on HIP
        # (di_head_prologue), never materialising the [2H, L1, L2] pair tensor T
        self.fuse_head_prologue = fuse_head_prologue
        # head_dtype / head_channels_last: the dilated-ResNet head's parameters and activations in
        # head_dtype (bf16: MIOpen bf16 convolutions, fp32 accumulation) and NHWC memory layout
        # (SURVEY §8f-3); the fp32 NCHW default is the parity configuration
        self.head_channels_last = head_channels_last
        # head_hip_ops: the head's InstanceNorm+ELU and SE-gate+residual passes on HIP
        # (head.HeadNormOps; NCHW only, so not with head_channels_last)
        self.head_hip_ops = head_hip_ops and not head_channels_last
        self.max_num_residues = max_num_residues
        self.interact_module = ResNet2DInputWithOptAttention(num_interact_layers, 2 * num_gnn_hidden_channels,
                                                             num_interact_hidden_channels, num_classes)
        self._geot_sd = None     # GeoT part of the reference state dict (host copy)
        self._prologue_w = None  # fp32 host copies of conv2d_1 / inorm_1 (fused head prologue)
        self._dev_ops = None     # (device, GeoTEngine, PairTensorOp, HeadPrologueOp | None)

    def load_reference_state_dict(self, sd):
        """Reference-keyed LitGINI state dict. The head loads into this nn.Module; the GeoT
        weights are kept on the host and packed for the GPU the model lives on at first use
        (so ``load`` on the CPU followed by ``.cuda()``, as lit_model_predict.py:214 does, works)."""
        head = {k[len("interact_module."):]: v for k, v in sd.items() if k.startswith("interact_module.")}
        self.interact_module.load_state_dict(head)
        self._geot_sd = {k: v.detach().to("cpu", copy=True) for k, v in sd.items()
                         if not k.startswith("interact_module.")}
        m = self.interact_module
        self._prologue_w = tuple(t.detach().to("cpu", torch.float32, copy=True) for t in
                                 (m.conv2d_1.weight, m.conv2d_1.bias, m.inorm_1.weight, m.inorm_1.bias))
        self._prologue_eps = m.inorm_1.eps
        self.interact_module.to(dtype=self.head_dtype)
        if self.head_channels_last:
            self.interact_module.to(memory_format=torch.channels_last)
        self._dev_ops = None
        return self

    def _ops(self):
        """(GeoTEngine, PairTensorOp, HeadPrologueOp | None) on the device of the model's
        parameters, (re)built when the model has moved. A model on the CPU raises: the kernels
        take device pointers only (no CPU fallback)."""
        if self._geot_sd is None:
            raise RuntimeError("load_reference_state_dict() / load_from_checkpoint() first")
        dev = gpu_device(next(self.interact_module.parameters()).device)
        if self._dev_ops is None or self._dev_ops[0] != dev:
            self._dev_ops = None
            eng = GeoTEngine(self._geot_sd, self.dtype, self.cfg, device=dev)
            pair = PairTensorOp(dev)
            pro = HeadPrologueOp(*self._prologue_w, self._prologue_eps, dev) if self.fuse_head_prologue else None
            self.interact_module.use_hip_norm_ops(HeadNormOps(dev) if self.head_hip_ops else None)
            self._dev_ops = (dev, eng, pair, pro)
        return self._dev_ops[1:]

    @property
    def engine(self):
        return self._ops()[0]

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location=None, strict=True, safe_globals=None, **kwargs):
        """LightningModule.load_from_checkpoint as lit_model_predict.py:214-219 calls it: build the
        network from the checkpoint's hyper-parameters (shapes inferred from the state dict where
        absent) and load its ``state_dict``. ``kwargs`` override hyper-parameters; the reference's
        training-only overrides (use_wandb_logger, batch_size, lr, weight_decay, dropout_rate) are
        accepted and have no effect on inference. The file is read with ``torch.load(weights_only=
        True)`` (``weights.read_checkpoint``). strict: every key this build needs must be present
        with its shape; keys outside node_in_embedding / gnn_module / interact_module are ignored."""
        from .weights import check_state_dict, infer_config, read_checkpoint
        sd, arch = read_checkpoint(checkpoint_path, safe_globals=safe_globals)
        net_prefixes = ("node_in_embedding.", "gnn_module.", "interact_module.")
        sd = type(sd)((k, v) for k, v in sd.items() if k.startswith(net_prefixes))
        arch.update({k: v for k, v in kwargs.items() if k in arch or k.startswith("num_") or k == "knn"})
        cfg = infer_config(sd, **arch)
        problems = check_state_dict(sd, cfg)
        if strict and problems:
            raise RuntimeError(f"{checkpoint_path}: state dict does not match LitGINI ({len(problems)} problems): "
                               + "; ".join(problems[:8]))
        opts = {k: kwargs[k] for k in ("dtype", "head_dtype", "precise_head", "fuse_head_prologue",
                                       "head_channels_last", "head_hip_ops") if k in kwargs}
        model = cls(num_node_input_feats=cfg.num_node_input_feats, num_gnn_layers=cfg.num_gnn_layers,
                    num_gnn_hidden_channels=cfg.num_gnn_hidden_channels,
                    num_gnn_attention_heads=cfg.num_gnn_attention_heads, knn=cfg.knn,
                    num_interact_layers=cfg.num_interact_layers,
                    num_interact_hidden_channels=cfg.num_interact_hidden_channels, num_classes=cfg.num_classes,
                    max_num_graph_nodes=cfg.node_count_limit,
                    max_num_residues=int(arch.get("max_num_residues", RESIDUE_COUNT_LIMIT)), **opts)
        if map_location is not None:
            model = model.to(map_location)
        return model.eval().load_reference_state_dict(sd)

    def freeze(self):
        """LightningModule.freeze (lit_model_predict.py:220): eval mode, no gradients."""
        for p in self.parameters():
            p.requires_grad_(False)
        return self.eval()

    # --- reference API ------------------------------------------------------------------
    def gnn_forward(self, graph):
        """node_in_embedding + GeoT for a (batched) graph; returns per-graph node features and
        writes ndata['f'] / edata['f'] like the reference (:1660-1679)."""
        graphs = _graph_list(graph)
        eng = self.engine
        gb = GraphBatch.from_graphs(graphs, device=eng.device, node_count_limit=self.cfg.node_count_limit)
        h, e = eng.forward(gb)
        graph.ndata["f"], graph.edata["f"] = h, e
        return [h[a:b] for a, b in zip(gb.node_off[:-1], gb.node_off[1:])]

    def interact_forward(self, interact_tensor, prologue_done=False):
        """Head on an interaction tensor; prologue_done: the input is already
        ELU(inorm_1(conv2d_1(T))) (HeadPrologueOp)."""
        x = interact_tensor.to(self.head_dtype)
        if self.head_channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        fn = self.interact_module.body if prologue_done else self.interact_module
        if self.precise_head:
            with torch.backends.cudnn.flags(enabled=False):
                return fn(x)
        return fn(x)

    def shared_step(self, graph1, graph2, return_representations=False):
        g1s, g2s = _graph_list(graph1), _graph_list(graph2)
        gb = GraphBatch.from_graphs(g1s + g2s, device=self.engine.device,
                                     node_count_limit=self.cfg.node_count_limit)
        logits_list, h, e = self._forward_batch(gb, [(i, len(g1s) + i) for i in range(len(g1s))])
        n1 = gb.node_off[len(g1s)]
        e1 = gb.edge_off[len(g1s)]
        graph1.ndata["f"], graph1.edata["f"] = h[:n1], e[:e1]
        graph2.ndata["f"], graph2.edata["f"] = h[n1:], e[e1:]
        if return_representations:
            np_ = lambda t: t.detach().float().cpu().numpy()  # noqa: E731
            return logits_list, np_(h[:n1]), np_(e[:e1]), np_(h[n1:]), np_(e[e1:])
        return logits_list

    def predict_step(self, batch, batch_idx=0, dataloader_idx=None):
        graph1, graph2 = batch[0], batch[1]
        return self.shared_step(graph1, graph2, return_representations=True)

    # --- batched entry ------------------------------------------------------------------
    def _forward_batch(self, gb: GraphBatch, pairs):
        eng, pair_op, prologue_op = self._ops()
        h, e = eng.forward(gb)
        off = gb.node_off
        h1r = [off[a] for a, _ in pairs]
        h2r = [off[b] for _, b in pairs]
        l1 = [gb.nodes_per_graph[a] for a, _ in pairs]
        l2 = [gb.nodes_per_graph[b] for _, b in pairs]
        if prologue_op is not None:
            _, views = prologue_op(h, h1r, h2r, l1, l2)
            logits = [self.interact_forward(v, prologue_done=True) for v in views]
        else:
            _, views = pair_op(h, h1r, h2r, l1, l2, hT=eng.last_hT)
            logits = [self.interact_forward(v) for v in views]
        return logits, h, e

    def predict_batch(self, gb: GraphBatch, pairs):
        """pairs: (chain-1 graph index, chain-2 graph index) per complex -> (logits, probs)."""
        logits, _, _ = self._forward_batch(gb, pairs)
        return logits, [contact_probs(lg) for lg in logits]


def construct_interact_tensor(graph1_feats, graph2_feats, pad=False, max_len=256):
    """deepinteract_utils.py:158-172 on the HIP pair-tensor kernel (pad=False path)."""
    if pad:
        raise NotImplementedError("pad=True (subsequencing) is disabled in the reference (:1699)")
    h = torch.cat([graph1_feats, graph2_feats]).contiguous()
    l1, l2 = graph1_feats.shape[0], graph2_feats.shape[0]
    _, views = PairTensorOp(h.device)(h, [0], [l1], [l1], [l2])
    return views[0]


__all__ = ["DGLGeometricTransformer", "LitGINI", "construct_interact_tensor", "batch_graphs", "unbatch"]
