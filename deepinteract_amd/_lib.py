"""ctypes binding of the C ABI in include/deepinteract_amd.h.

The product path has no fallback: if the HIP library cannot be loaded every op raises.
"""
from __future__ import annotations

import ctypes
import os

from . import build as _build

DI_F32, DI_BF16 = 0, 1


class DiGraph(ctypes.Structure):
    _fields_ = [("num_nodes", ctypes.c_int32), ("num_edges", ctypes.c_int32),
                ("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("nbr", ctypes.c_void_p),
                ("node_pos", ctypes.c_void_p), ("in_ptr", ctypes.c_void_p), ("flags", ctypes.c_int32)]


DI_GRAPH_GEO_REF = 1


class DiGeoArgs(ctypes.Structure):
    _fields_ = [("num_graphs", ctypes.c_int32), ("k", ctypes.c_int32), ("max_nodes", ctypes.c_int32),
                ("node_off", ctypes.c_void_p), ("backbone", ctypes.c_void_p), ("amide_norm", ctypes.c_void_p),
                ("dips", ctypes.c_void_p), ("knn_idx", ctypes.c_void_p), ("knn_d2", ctypes.c_void_p),
                ("node_f", ctypes.c_void_p), ("edge_f", ctypes.c_void_p), ("stats", ctypes.c_void_p)]


class DiPairDesc(ctypes.Structure):
    _fields_ = [("h1_row", ctypes.c_int64), ("h2_row", ctypes.c_int64), ("out_off", ctypes.c_int64),
                ("l1", ctypes.c_int32), ("l2", ctypes.c_int32)]


class DiPairLaunch(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_int32), ("blocks", ctypes.c_int32), ("waves_per_block", ctypes.c_int32),
                ("beside", ctypes.c_int32)]


DI_PAIR_AUTO, DI_PAIR_ROWS, DI_PAIR_VECTOR, DI_PAIR_LINES = 0, 1, 2, 3
ABI_VERSION = 8


class DiPairJob(ctypes.Structure):
    _fields_ = [("hT", ctypes.c_void_p), ("descs", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("num_rows", ctypes.c_int32), ("num_complexes", ctypes.c_int32), ("max_l1", ctypes.c_int32),
                ("items", ctypes.c_int32)]


# pair-queue words (include/deepinteract_amd.h, di_pair_queue_bytes)
PQ_READY, PQ_ERROR, PQ_GAVE_UP, PQ_SBYTES, PQ_HBYTES = 0, 32, 33, 40, 42


_P = ctypes.c_void_p
_I = ctypes.c_int32
_SIGS = {
    "di_abi_version": ([], ctypes.c_int),
    "di_blob_bytes": ([ctypes.c_int, ctypes.c_int, ctypes.c_int], ctypes.c_int64),
    "di_blob_layout": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "di_node_embed": ([ctypes.POINTER(DiGraph), _I, _I, _P, _P, _P, _P, _P, _P, _I, _P], ctypes.c_int),
    "di_init_edge": ([ctypes.POINTER(DiGraph), _I, _P, _P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
    "di_init_edge_resident": ([ctypes.POINTER(DiGraph), _P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
    "di_embed_init_edge": ([ctypes.POINTER(DiGraph), _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P],
                           ctypes.c_int),
    "di_edge_layer": ([ctypes.POINTER(DiGraph), _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
                      ctypes.c_int),
    "di_node_layer": ([ctypes.POINTER(DiGraph), _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
    "di_node_aggregate": ([ctypes.POINTER(DiGraph), _I, _P, _P, _P, _P], ctypes.c_int),
    "di_node_update": ([ctypes.POINTER(DiGraph), _I, _I, _P, _P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
    "di_attn_parts_bytes": ([_I], ctypes.c_int64),
    "di_edge_layer_attn": ([ctypes.POINTER(DiGraph), _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
                           ctypes.c_int),
    "di_node_update_folded": ([ctypes.POINTER(DiGraph), _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
    "di_pair_tensor": ([_I, _P, _I, _I, _I, _I, _I, _P, _P, _I, ctypes.POINTER(DiPairLaunch), _P, _P], ctypes.c_int),
    "di_pair_tensor_check": ([_I, _I, _I, _I, _I, ctypes.POINTER(DiPairLaunch)], ctypes.c_int),
    "di_pair_queue_bytes": ([_I], ctypes.c_int64),
    "di_pair_job_items": ([_I, _I, _I], ctypes.c_int32),
    "di_pair_signal": ([_P, _I, _P], ctypes.c_int),
    "di_pair_stream": ([_I, _P, _I, _I, _I, _P, ctypes.POINTER(DiPairLaunch), ctypes.c_float, _P], ctypes.c_int),
    "di_pair_help": ([_I, _P, _I, _I, _I, _P, ctypes.POINTER(DiPairLaunch), _I, _P], ctypes.c_int),
    "di_stream_create_dedicated": ([ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "di_stream_destroy": ([_P], ctypes.c_int),
    "di_streams_concurrent": ([_P, _P, _P, ctypes.c_float, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "di_head_prologue": ([_I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, ctypes.c_float, _P, _P, _P],
                         ctypes.c_int),
    "di_head_prologue_work_bytes": ([_I, _I, _I, _I], ctypes.c_int64),
    "di_inorm_elu": ([_I, _P, _I, ctypes.c_int64, _P, _P, ctypes.c_float, _P, _P, _P], ctypes.c_int),
    "di_inorm_work_bytes": ([_I, ctypes.c_int64], ctypes.c_int64),
    "di_se_scale_add": ([_I, _P, _P, _P, _P, _I, ctypes.c_int64, _P, _P], ctypes.c_int),
    "di_channel_mean": ([_I, _P, _I, ctypes.c_int64, _P, _P, _P, _P], ctypes.c_int),
    "di_knn_topk": ([_I, _P, _P, _I, _I, _P, _P, _P], ctypes.c_int),
    "di_geo_feats": ([ctypes.POINTER(DiGeoArgs), _P], ctypes.c_int),
    "di_build_nbr_ids": ([_I, _P, _P, _P, ctypes.c_uint64, _P, _P], ctypes.c_int),
    "di_build_nbr_ids_torch": ([_I, _P, _I, _P, _I, _P, _P, _P, _P], ctypes.c_int),
    "di_knn_graph": ([_I, _P, _I, _P, _I, _P, _P, _P, _P, _P], ctypes.c_int),
    "di_conformation": ([ctypes.POINTER(DiGraph), _I, _P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
    "di_gemm_bias_act": ([_I, _I, _I, _I, _P, _I, _P, _P, _I, _P, _I, _P, _I, _P], ctypes.c_int),
    "di_geo_attention": ([ctypes.POINTER(DiGraph), _I, _P, _P, _P, _P, _P, _P], ctypes.c_int),
}

_lib = None


def library_path() -> str:
    return _build.LIB


def _bind(path: str):
    lib = ctypes.CDLL(path)
    for name, (argtypes, restype) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    if lib.di_abi_version() != ABI_VERSION:
        raise RuntimeError("deepinteract_amd ABI version mismatch")
    return lib


def load(build_if_missing: bool = True):
    """Load (building first if needed) the in-tree HIP library; raises if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    # torch ships its own libamdhip64.so.7: load it first so this library binds to the SAME HIP
    # runtime (same SONAME) instead of pulling /opt/rocm's copy into the process.
    import torch  # noqa: F401
    if not os.path.exists(_build.LIB) or (build_if_missing and not _build.up_to_date()):
        if not build_if_missing:
            raise RuntimeError(f"deepinteract_amd HIP library missing: {_build.LIB}")
        _build.build()
    _lib = _bind(_build.LIB)
    return _lib


def load_variant(path: str):
    """Tuning only (bench.py --lib): bind a launch-shape variant of the library built by
    build.build_variant() instead of the in-tree one. Must run before any other load()."""
    global _lib
    if _lib is not None:
        raise RuntimeError("the HIP library is already loaded")
    import torch  # noqa: F401
    if not os.path.exists(path):
        raise RuntimeError(f"variant library {path} does not exist")
    _lib = _bind(path)
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")
