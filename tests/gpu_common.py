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


def rel_elem(a, b, floor=0.0):
    """Elementwise relative error max |a - b| / max(|b|, floor) (north_star's "<= 1e-4 relative"
    read per element; rel_max is the normwise figure). floor > 0 only for signed features whose
    reference values cross zero; contact probabilities (in (0, 1)) use none."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float((np.abs(a - b) / np.maximum(np.abs(b), floor)).max())
