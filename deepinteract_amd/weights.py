"""Seeded, reproducible LitGINI weights under the reference's state-dict key names.

No trained checkpoint exists offline (Zenodo, README.md:249-252), so parity runs on seeded
weights. Each tensor is drawn from its own ``torch.Generator('cpu')`` seeded from
``(seed, crc32(key))``: the values do not depend on key order and are identical on any host
(torch's CPU Mersenne-Twister is platform independent). BatchNorm running stats and affine
parameters are randomised so that every folded BatchNorm is non-trivial.

Key layout mirrors ``LitGINI`` (deepinteract_modules.py:1478-1625), including the ResBlock
quirk that ONE BatchNorm1d instance is registered three times (``res_block.1/.4/.7``,
deepinteract_modules.py:468-479): the three keys always carry identical values.
"""
from __future__ import annotations

import hashlib
import math
import re
import zlib
from collections import OrderedDict

import numpy as np
import torch

from .config import GeoTConfig, NUM_RBF


def _linear(keys, name, out_f, in_f, bias):
    keys.append((f"{name}.weight", (out_f, in_f), "lin_w"))
    if bias:
        keys.append((f"{name}.bias", (out_f,), "bias"))


def _bn(keys, name, c):
    keys.append((f"{name}.weight", (c,), "bn_w"))
    keys.append((f"{name}.bias", (c,), "bn_b"))
    keys.append((f"{name}.running_mean", (c,), "bn_mean"))
    keys.append((f"{name}.running_var", (c,), "bn_var"))
    keys.append((f"{name}.num_batches_tracked", (), "bn_nbt"))


def _conf_keys(keys, p, cfg: GeoTConfig):
    H, S, G = cfg.num_gnn_hidden_channels, cfg.shared_embed_size, cfg.geo_embed_size
    _linear(keys, f"{p}.dist_linear_0", G, NUM_RBF, False)
    _linear(keys, f"{p}.dist_linear_1", H, G, False)
    _linear(keys, f"{p}.dir_linear_0", G, 3, False)
    _linear(keys, f"{p}.dir_linear_1", S, G, False)
    _linear(keys, f"{p}.orient_linear_0", G, 4, False)
    _linear(keys, f"{p}.orient_linear_1", S, G, False)
    _linear(keys, f"{p}.amide_linear_0", G, 1, False)
    _linear(keys, f"{p}.amide_linear_1", S, G, False)
    _linear(keys, f"{p}.nbr_linear", H, H, True)
    _linear(keys, f"{p}.orig_msg_linear", H, H, True)
    _linear(keys, f"{p}.downward_proj", S, H, False)
    _linear(keys, f"{p}.upward_proj", H, S, False)
    _linear(keys, f"{p}.res_connect_linear", H, H, True)
    for kind, n in (("pre_res_blocks", cfg.num_pre_res_blocks), ("post_res_blocks", cfg.num_post_res_blocks)):
        for b in range(n):
            rb = f"{p}.{kind}.{b}.res_block"
            for i in (0, 3, 6):
                _linear(keys, f"{rb}.{i}", H, H, True)
                _bn(keys, f"{rb}.{i + 1}", H)
    _linear(keys, f"{p}.final_dist_linear", H, NUM_RBF, False)
    _linear(keys, f"{p}.final_dir_linear", H, 3, False)
    _linear(keys, f"{p}.final_orient_linear", H, 4, False)
    _linear(keys, f"{p}.final_amide_linear", H, 1, False)
    _linear(keys, f"{p}.final_linear", H, H, True)


def geot_keys(cfg: GeoTConfig = GeoTConfig()):
    """(key, shape, kind) for node_in_embedding + gnn_module.0 (DGLGeometricTransformer)."""
    H = cfg.num_gnn_hidden_channels
    keys = []
    _linear(keys, "node_in_embedding", H, cfg.num_node_input_feats, False)
    ie = "gnn_module.0.init_edge_module"
    keys.append((f"{ie}.node_embedding.weight", (cfg.node_count_limit, H), "emb"))
    for suffix in ("0", "1"):
        _linear(keys, f"{ie}.edge_messages_linear_{suffix}", H, 2, False)
        _linear(keys, f"{ie}.dist_linear_{suffix}", H, NUM_RBF, False)
        _linear(keys, f"{ie}.dir_linear_{suffix}", H, 3, False)
        _linear(keys, f"{ie}.orient_linear_{suffix}", H, 4, False)
        _linear(keys, f"{ie}.amide_linear_{suffix}", H, 1, False)
        if suffix == "0":
            _linear(keys, f"{ie}.combined_linear_0", H, 7 * H, False)
    _linear(keys, f"{ie}.combined_linear_1", 28, H, False)
    _linear(keys, f"{ie}.combined_linear_2", H, 28, False)
    L = cfg.num_gnn_layers
    for li in range(L):
        p = f"gnn_module.0.gt_block.{li}"
        final = li == L - 1
        _conf_keys(keys, f"{p}.conformation_module", cfg)
        _bn(keys, f"{p}.batch_norm1_node_feats", H)
        _bn(keys, f"{p}.batch_norm1_edge_feats", H)
        for q in ("Q", "K", "V", "edge_feats_projection"):
            _linear(keys, f"{p}.mha_module.{q}", H, H, False)
        _linear(keys, f"{p}.O_node_feats", H, H, True)
        if not final:
            _linear(keys, f"{p}.O_edge_feats", H, H, True)
        _linear(keys, f"{p}.node_feats_MLP.0", 2 * H, H, False)
        _linear(keys, f"{p}.node_feats_MLP.3", H, 2 * H, False)
        _bn(keys, f"{p}.batch_norm2_node_feats", H)
        if not final:
            _bn(keys, f"{p}.batch_norm2_edge_feats", H)
            _linear(keys, f"{p}.edge_feats_MLP.0", 2 * H, H, False)
            _linear(keys, f"{p}.edge_feats_MLP.3", H, 2 * H, False)
    return keys


def _conv(keys, name, o, i, k):
    keys.append((f"{name}.weight", (o, i, k, k), "conv_w"))
    keys.append((f"{name}.bias", (o,), "conv_b"))


def _inorm(keys, name, c):
    keys.append((f"{name}.weight", (c,), "bn_w"))
    keys.append((f"{name}.bias", (c,), "bn_b"))


def head_keys(cfg: GeoTConfig = GeoTConfig()):
    """(key, shape, kind) for interact_module = ResNet2DInputWithOptAttention
    (deepinteract_modules.py:1155-1248, ResNet :973-1106, SEBlock :954-970)."""
    C, H = cfg.num_interact_hidden_channels, cfg.num_gnn_hidden_channels
    keys = []
    p = "interact_module"
    _conv(keys, f"{p}.conv2d_1", C, 2 * H, 1)
    _inorm(keys, f"{p}.inorm_1", C)

    def resnet(prefix, mname, chunks, inorm, extra):
        _conv(keys, f"{prefix}.resnet_{mname}_init_proj", C, C, 1)
        blocks = [f"{i}_{d}" for i in range(chunks) for d in (1, 2, 4, 8)]
        if extra:
            blocks += ["extra0", "extra1"]
        for b in blocks:
            r = f"{prefix}.resnet_{mname}_{b}"
            if inorm:
                _inorm(keys, f"{r}_inorm_1", C)
                _inorm(keys, f"{r}_inorm_2", C // 2)
                _inorm(keys, f"{r}_inorm_3", C // 2)
            _conv(keys, f"{r}_conv2d_1", C // 2, C, 1)
            _conv(keys, f"{r}_conv2d_2", C // 2, C // 2, 3)
            _conv(keys, f"{r}_conv2d_3", C, C // 2, 1)
            _linear(keys, f"{r}_se_block.linear1", C // 16, C, True)
            _linear(keys, f"{r}_se_block.linear2", C, C // 16, True)

    resnet(f"{p}.base_resnet", "base_resnet", cfg.num_interact_layers, True, False)
    resnet(f"{p}.phase2_resnet", "bin_resnet", 1, False, True)
    _conv(keys, f"{p}.phase2_conv", cfg.num_classes, C, 1)
    return keys


def _canonical_key(key: str) -> str:
    # the shared ResBlock BatchNorm: .4 and .7 alias .1
    for alias in (".res_block.4.", ".res_block.7."):
        if alias in key:
            return key.replace(alias, ".res_block.1.")
    return key


def _draw(key: str, shape, kind: str, seed: int) -> torch.Tensor:
    g = torch.Generator(device="cpu")
    g.manual_seed((seed * 1_000_003 + zlib.crc32(_canonical_key(key).encode())) % (2 ** 63))

    def u(lo, hi):
        return lo + (hi - lo) * torch.rand(shape, generator=g, dtype=torch.float64)

    if kind == "lin_w":
        out_f, in_f = shape
        b = math.sqrt(6.0 / (in_f + out_f))
        t = u(-b, b)
    elif kind == "bias":
        t = u(-0.1, 0.1)
    elif kind == "bn_w":
        t = u(0.8, 1.2)
    elif kind == "bn_b":
        t = u(-0.1, 0.1)
    elif kind == "bn_mean":
        t = u(-0.2, 0.2)
    elif kind == "bn_var":
        t = u(0.6, 1.4)
    elif kind == "bn_nbt":
        return torch.tensor(0, dtype=torch.long)
    elif kind == "emb":
        t = u(-math.sqrt(3.0), math.sqrt(3.0))
    elif kind in ("conv_w", "conv_b"):
        fan_in = None
        t = None
        if kind == "conv_w":
            fan_in = shape[1] * shape[2] * shape[3]
        else:
            fan_in = shape[0]  # bias bound uses the weight's fan-in below
        b = 1.0 / math.sqrt(fan_in)
        t = u(-b, b)
    else:
        raise ValueError(kind)
    return t.to(torch.float32)


def glorot_orthogonal(tensor: torch.Tensor, scale: float, generator=None) -> torch.Tensor:
    """deepinteract_utils.py:47-52: orthogonal_ then W *= sqrt(scale / ((fan_out + fan_in) * var(W)))."""
    torch.nn.init.orthogonal_(tensor, generator=generator)
    s = scale / ((tensor.size(-2) + tensor.size(-1)) * tensor.var())
    tensor.mul_(s.sqrt())
    return tensor


def reference_init_state_dict(seed: int = 0, cfg: GeoTConfig = GeoTConfig(), with_head: bool = True):
    """A LitGINI state dict initialised the way the reference's modules initialise themselves
    (SURVEY.md §8a a14), from one seeded CPU generator:
      * every GeoT linear weight: glorot_orthogonal(scale=2.0) (reset_parameters at
        deepinteract_modules.py:55-74, 176-196, 336-371, 483-490, 652-667, 879-890, 1585-1589),
        their biases zero-filled; BatchNorm at its defaults (1, 0, running 0 / 1);
      * InitEdge's positional nn.Embedding: U(-sqrt(3), sqrt(3)) (:179);
      * the head: PyTorch's default Conv2d / Linear init (U(+-1/sqrt(fan_in)) for weights and biases),
        InstanceNorm affine at (1, 0), and phase2_conv.bias[1] = -7 (:1221-1226).
    The values are not the reference's own random draws (torch's RNG stream over its module
    construction order is not reproduced); the distributions and the deterministic parts are."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    sd = OrderedDict()
    shared = {}
    keys = geot_keys(cfg) + (head_keys(cfg) if with_head else [])
    for key, shape, kind in keys:
        canon = _canonical_key(key)
        if canon in shared:  # the ResBlock's one BatchNorm, registered three times
            sd[key] = shared[canon].clone()
            continue
        head = key.startswith("interact_module.")
        if kind == "bn_nbt":
            t = torch.tensor(0, dtype=torch.long)
        elif kind in ("bn_w", "bn_var"):
            t = torch.ones(shape)
        elif kind in ("bn_b", "bn_mean"):
            t = torch.zeros(shape)
        elif kind == "emb":
            t = torch.empty(shape).uniform_(-math.sqrt(3.0), math.sqrt(3.0), generator=g)
        elif kind == "lin_w" and not head:
            t = glorot_orthogonal(torch.empty(shape), 2.0, generator=g)
        elif kind == "bias" and not head:
            t = torch.zeros(shape)
        elif kind in ("lin_w", "conv_w"):
            fan_in = int(np.prod(shape[1:]))
            b = 1.0 / math.sqrt(fan_in)
            t = torch.empty(shape).uniform_(-b, b, generator=g)
        elif kind in ("bias", "conv_b"):
            w_shape = next(s for k, s, _ in keys if k == key[:-len("bias")] + "weight")
            b = 1.0 / math.sqrt(int(np.prod(w_shape[1:])))
            t = torch.empty(shape).uniform_(-b, b, generator=g)
        else:
            raise ValueError(kind)
        if key == "interact_module.phase2_conv.bias":
            t[1] = -7.0
        sd[key] = shared[canon] = t.to(torch.float32) if t.is_floating_point() else t
    return sd


def seeded_state_dict(seed: int = 0, cfg: GeoTConfig = GeoTConfig(), with_head: bool = True):
    """Reference-keyed LitGINI state dict with seeded values (fp32, CPU)."""
    sd = OrderedDict()
    keys = geot_keys(cfg) + (head_keys(cfg) if with_head else [])
    for key, shape, kind in keys:
        sd[key] = _draw(key, shape, kind, seed)
    return sd


def state_dict_sha256(sd) -> str:
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


# hyper-parameters of the reference LitGINI (deepinteract_modules.py:1481-1489) that shape the
# inference network; everything else in a checkpoint's hyper_parameters (optimiser, logging,
# training flags) has no effect on predict.
_ARCH_HPARAMS = ("num_node_input_feats", "num_gnn_layers", "num_gnn_hidden_channels", "num_gnn_attention_heads",
                 "knn", "num_interact_layers", "num_interact_hidden_channels", "num_classes",
                 "max_num_graph_nodes", "max_num_residues")


def read_checkpoint(path, safe_globals=None):
    """A PyTorch-Lightning checkpoint of the reference LitGINI (as lit_model_predict.py:214 loads
    it) -> (state_dict, architecture hparams). Loaded with ``torch.load(weights_only=True)``
    only: nothing in the file is executed. The reference saves ``gnn_activ_fn=nn.SiLU()`` among
    its hyper-parameters, so ``torch.nn.SiLU`` is allow-listed for the weights-only unpickler;
    a file that needs any other global is refused (extract its ``state_dict`` first)."""
    allowed = [torch.nn.SiLU] + list(safe_globals or [])
    with torch.serialization.safe_globals(allowed):
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(ckpt, dict) and "state_dict" in ckpt:
        sd, hp = ckpt["state_dict"], dict(ckpt.get("hyper_parameters") or {})
    elif isinstance(ckpt, dict) and all(isinstance(v, torch.Tensor) for v in ckpt.values()):
        sd, hp = ckpt, {}  # a bare state dict
    else:
        raise ValueError(f"{path}: neither a Lightning checkpoint nor a state dict")
    arch = {k: hp[k] for k in _ARCH_HPARAMS if k in hp and isinstance(hp[k], (int, float))}
    return OrderedDict((k, v) for k, v in sd.items()), arch


def infer_config(sd, **overrides) -> GeoTConfig:
    """GeoTConfig from a reference-keyed state dict's shapes (node_in_embedding, gt_block count,
    base_resnet chunk count), overridden by explicit hyper-parameters."""
    w = sd["node_in_embedding.weight"]
    layers = {int(k.split(".")[3]) for k in sd if k.startswith("gnn_module.0.gt_block.")}
    pat = re.compile(r"^interact_module\.base_resnet\.resnet_base_resnet_(\d+)_(?:1|2|4|8)_")
    chunks = {int(m.group(1)) for m in map(pat.match, sd) if m}
    kw = dict(num_node_input_feats=int(w.shape[1]), num_gnn_hidden_channels=int(w.shape[0]),
              num_gnn_layers=len(layers) or GeoTConfig().num_gnn_layers)
    if chunks:
        kw["num_interact_layers"] = max(chunks) + 1
    pos = sd.get("gnn_module.0.init_edge_module.node_embedding.weight")
    if pos is not None:  # nn.Embedding(max_num_graph_nodes, H) (deepinteract_modules.py:153)
        kw["node_count_limit"] = int(pos.shape[0])
    for k in ("num_gnn_attention_heads", "knn", "num_interact_hidden_channels", "num_classes",
              "num_node_input_feats", "num_gnn_layers", "num_gnn_hidden_channels", "num_interact_layers"):
        if k in overrides:
            kw[k] = int(overrides[k])
    if "max_num_graph_nodes" in overrides:
        kw["node_count_limit"] = int(overrides["max_num_graph_nodes"])
    return GeoTConfig(**kw)


def check_state_dict(sd, cfg: GeoTConfig, with_head: bool = True):
    """Strict key / shape check of a reference-keyed state dict against this build's layout
    (geot_keys + head_keys). Returns the list of problems (empty when it matches)."""
    want = {k: shape for k, shape, _ in geot_keys(cfg) + (head_keys(cfg) if with_head else [])}
    problems = [f"missing {k}" for k in want if k not in sd]
    problems += [f"unexpected {k}" for k in sd if k not in want]
    problems += [f"shape {k}: {tuple(sd[k].shape)} != {tuple(s)}" for k, s in want.items()
                 if k in sd and tuple(sd[k].shape) != tuple(s)]
    return problems
