"""Shared helpers for the GPU parity tests (fixtures -> device batches)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_case(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


def chain_item(z, tag):
    return {
        "num_nodes": int(z[f"{tag}_node_f"].shape[0]),
        "src": torch.as_tensor(z[f"{tag}_src"]).long(),
        "dst": torch.as_tensor(z[f"{tag}_dst"]).long(),
        "src_nbr": torch.as_tensor(z[f"{tag}_src_nbr"]).long(),
        "dst_nbr": torch.as_tensor(z[f"{tag}_dst_nbr"]).long(),
        "node_f": torch.as_tensor(z[f"{tag}_node_f"]),
        "edge_f": torch.as_tensor(z[f"{tag}_edge_f"]),
    }


def chain_arrays(z, tag):
    return {k: z[f"{tag}_{k}"] for k in ("backbone", "amide_norm", "dips")}


def rel_max(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def logit_floor(ref):
    """The denominator floor rel_elem uses for logits: none when the reference logits keep one sign,
    else 1e-3 of the largest |reference logit| (elements that cross zero have no meaningful relative
    error below that)."""
    ref = np.asarray(ref)
    return 1e-3 * float(np.abs(ref).max()) if ref.min() < 0.0 < ref.max() else 0.0


def close_elem(a, b, rtol=1e-4, atol_frac=1e-5):
    """Worst element of |a - b| / (rtol |b| + atol_frac max|b|) (numpy.allclose's form; <= 1 passes).
    The logits' elementwise bar: fp32 accumulation-order differences leave an absolute error of a
    few 1e-6 on every logit, which dominates the relative error of logits that cross zero (measured
    on MI355X, DESIGN.md section 2: floored relative 1.7e-3..1.9e-3, absolute <= 4e-6 on max|b| ~ 2)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float((np.abs(a - b) / (rtol * np.abs(b) + atol_frac * np.abs(b).max())).max())


def rel_elem(a, b, floor=0.0):
    """Elementwise relative error max |a - b| / max(|b|, floor) (north_star's "<= 1e-4 relative"
    read per element; rel_max is the normwise figure). floor > 0 only for signed features whose
    reference values cross zero; contact probabilities (in (0, 1)) use none."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float((np.abs(a - b) / np.maximum(np.abs(b), floor)).max())
