"""CU-masked HIP streams: spatial partitioning of the GPU between the compute-bound GeoT kernels
and the HBM-store-bound pair-tensor kernel.

The pair tensor is a pure store stream that 32-64 CUs alone drive at 3.4-5.6 TB/s; sharing every
CU with the GeoT edge kernels instead slows both (their LDS-DMA weight streams queue behind the
stores). `hipExtStreamCreateWithCUMask` gives each stream its own CU set; torch adopts the
streams with `torch.cuda.ExternalStream`.
"""
from __future__ import annotations

import ctypes
import glob
import os

import torch

_hip = None


def _hip_lib():
    """The HIP runtime torch already loaded (same SONAME, same process-wide runtime)."""
    global _hip
    if _hip is None:
        cands = sorted(glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*")))
        _hip = ctypes.CDLL(cands[0] if cands else "libamdhip64.so")
        _hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
        _hip.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
    return _hip


def split_cus(num_cus: int, k: int, layout: str = "stride"):
    """(pair CUs, GeoT CUs): k CUs for the store stream, the rest for GeoT. layout "stride"
    spreads the k CUs evenly over the CU index space (every num_cus/k-th), "contig" takes
    the first k."""
    if not 0 < k < num_cus:
        raise ValueError(f"k={k} must be in 1..{num_cus - 1}")
    if layout == "contig":
        pair = list(range(k))
    else:
        step = num_cus / k
        pair = sorted({int(i * step) for i in range(k)})
    rest = [c for c in range(num_cus) if c not in set(pair)]
    return pair, rest


def cu_mask_words(cus, num_cus: int):
    words = [0] * ((num_cus + 31) // 32)
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    return words


def masked_stream(device, cus, num_cus: int) -> torch.cuda.ExternalStream:
    """A new HIP stream restricted to the CU indices `cus`, as a torch stream."""
    with torch.cuda.device(device):
        words = cu_mask_words(cus, num_cus)
        arr = (ctypes.c_uint32 * len(words))(*words)
        ptr = ctypes.c_void_p()
        rc = _hip_lib().hipExtStreamCreateWithCUMask(ctypes.byref(ptr), len(words), arr)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
        return torch.cuda.ExternalStream(ptr.value, device=device)
