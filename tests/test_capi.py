"""The C-ABI library builds for gfx950, loads, and exports every entry point that
include/deepinteract_amd.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

from deepinteract_amd import _lib, build, packing

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "deepinteract_amd.h")).read()
    return sorted(set(re.findall(r"\b(di_[a-z0-9_]+)\s*\(", src)))


def test_library_builds_and_exports_all_declared_symbols():
    path = build.build()
    lib = ctypes.CDLL(path)
    syms = declared_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(lib, s), s


def test_abi_version_and_blob_sizes():
    lib = _lib.load()
    assert lib.di_abi_version() == _lib.ABI_VERSION == 8
    for kind, (nblk, nvec) in packing.BLOB_SIZES.items():
        assert lib.di_blob_bytes(kind, _lib.DI_F32, 0) == nblk * 512 * 4
        assert lib.di_blob_bytes(kind, _lib.DI_BF16, 0) == nblk * 512 * 2
        assert lib.di_blob_bytes(kind, _lib.DI_F32, 1) == nvec * 4
    assert lib.di_blob_bytes(9, _lib.DI_F32, 0) == -1
    # fragment order (ABI 5): the bf16 edge-layer blobs are packed for v_mfma_f32_32x32x16_bf16
    for kind in range(7):
        assert lib.di_blob_layout(kind, _lib.DI_F32) == 16
        assert lib.di_blob_layout(kind, _lib.DI_BF16) == (32 if kind in (1, 2, 3) else 16)
    assert lib.di_blob_layout(7, _lib.DI_BF16) == -1 and lib.di_blob_layout(2, 5) == -1


def test_invalid_arguments_rejected_without_gpu():
    lib = _lib.load()
    assert lib.di_node_embed(None, 0, 113, None, None, None, None, None, None, -1, None) == -1
    assert lib.di_pair_tensor(0, None, 0, 0, 0, 128, 1, None, None, 0, None, None, None) == -1
    assert lib.di_knn_topk(1, None, None, 20, 10, None, None, None) == -1
    assert lib.di_head_prologue(0, None, 1, 8, 8, 128, 128, 1, None, None, None, None, None, 1e-6,
                                None, None, None) == -1


def test_pair_tensor_check_shapes_and_launch():
    """di_pair_tensor's host-side validation (di_pair_tensor_check), without a GPU: the model limit
    4096 x 4096 (plane = 2^24 elements, refused with DI_ERANGE in round 2) passes in both dtypes;
    planes of 2^31 bytes and more, and more than 2^20 rows, are DI_ERANGE; bad launches DI_EINVAL."""
    import ctypes
    lib = _lib.load()
    L = _lib.DiPairLaunch
    assert lib.di_pair_tensor_check(1, 4096, 4096, 128, 2, None) == 0
    assert lib.di_pair_tensor_check(8, 4096, 4096, 128, 4, None) == 0
    assert lib.di_pair_tensor_check(64, 1000, 1000, 128, 2, None) == 0
    assert lib.di_pair_tensor_check(1, 32768, 32768, 128, 2, None) == -2   # 2 GiB plane
    assert lib.di_pair_tensor_check(1, 1 << 21, 8, 128, 2, None) == -2     # row index range
    assert lib.di_pair_tensor_check(0, 10, 10, 128, 2, None) == -1
    assert lib.di_pair_tensor_check(1, 10, 10, 128, 3, None) == -1
    for launch, rc in ((L(_lib.DI_PAIR_LINES, 0, 2, 1), 0), (L(4, 0, 0, 0), -1), (L(-1, 0, 0, 0), -1),
                       (L(0, -1, 0, 0), -1), (L(0, 0, 17, 0), -1), (L(0, 0, 0, 2), -1)):
        assert lib.di_pair_tensor_check(1, 64, 64, 128, 2, ctypes.byref(launch)) == rc, (launch.kernel, rc)
    # the lines kernel needs 128-B aligned planes (aligned == 2), rows / vector 16-B ones: refused
    # before any launch (dummy non-NULL pointers are never dereferenced on these paths)
    p = ctypes.c_void_p(16)
    for kernel, aligned in ((_lib.DI_PAIR_LINES, 1), (_lib.DI_PAIR_ROWS, 0), (_lib.DI_PAIR_VECTOR, 0)):
        launch = L(kernel, 0, 0, 0)
        assert lib.di_pair_tensor(1, p, 1, 64, 64, 128, aligned, p, p, 128, ctypes.byref(launch), p, None) == -1
    assert lib.di_pair_tensor(1, p, 1, 64, 64, 128, 3, p, p, 128, None, p, None) == -1
    assert lib.di_pair_tensor(1, p, 1, 64, 64, 128, 1, p, None, 128, None, p, None) == -1  # aligned needs hT


def test_geo_ref_fn_contract_without_gpu():
    """Fn rows may be omitted (NULL) only for DI_GRAPH_GEO_REF batches: without the flag the
    kernels need them and the entry points refuse NULL before any launch (dummy non-NULL
    pointers are never dereferenced on these paths)."""
    import ctypes
    lib = _lib.load()
    p = ctypes.c_void_p(16)
    g = _lib.DiGraph(8, 16, 16, 16, 16, 16, 16, 0)
    assert lib.di_init_edge(ctypes.byref(g), _lib.DI_BF16, p, p, p, p, p, p, None, None) == -1
    # the resident InitEdge is the DI_GRAPH_GEO_REF path only
    assert lib.di_init_edge_resident(ctypes.byref(g), p, p, p, p, p, p, None) == -1
    assert lib.di_embed_init_edge(ctypes.byref(g), _lib.DI_BF16, 113, p, p, p, p, p, p, p, p, p, p, p, None, -1, None) == -1
    assert lib.di_embed_init_edge(ctypes.byref(g), _lib.DI_F32, 113, p, p, p, p, p, p, p, p, p, p, p, None, -1, None) == -1
    assert lib.di_edge_layer(ctypes.byref(g), _lib.DI_BF16, 0, p, p, None, p, p, p, p, p, p, None) == -1
    assert lib.di_edge_layer(ctypes.byref(g), _lib.DI_BF16, 0, p, p, p, p, p, p, p, p, None, None) == -1
    assert _lib.DI_GRAPH_GEO_REF == 1


def test_head_prologue_work_bytes():
    lib = _lib.load()
    # per (complex, channel): a', b', e^a', e^b' fp32 tables + one int32 flag
    assert lib.di_head_prologue_work_bytes(8, 1000, 900, 128) == 8 * 128 * (2 * 1900 * 4 + 4)
    assert lib.di_head_prologue_work_bytes(0, 10, 10, 128) == 0


def test_ctypes_struct_layouts():
    assert ctypes.sizeof(_lib.DiGraph) == 8 + 5 * 8 + 8  # + int32 flags, padded to 8
    assert ctypes.sizeof(_lib.DiPairDesc) == 32
    assert ctypes.sizeof(_lib.DiGeoArgs) == 16 + 8 * 9
    assert ctypes.sizeof(_lib.DiPairJob) == 3 * 8 + 4 * 4


def test_pair_queue_host_contract():
    """The pair queue's sizes and argument validation (host only, no launch): 256 B of header plus
    256 B per job; items = complexes x 2H x ceil(L1 / 64); refusals before any launch."""
    lib = _lib.load()
    assert lib.di_pair_queue_bytes(1) == 256 + 256
    assert lib.di_pair_queue_bytes(128) == 256 * 129
    assert lib.di_pair_queue_bytes(0) == -1
    assert lib.di_pair_job_items(8, 1000, 128) == 8 * 256 * 16
    assert lib.di_pair_job_items(2, 4000, 128) == 2 * 256 * 63
    assert lib.di_pair_job_items(0, 1000, 128) == -1
    assert lib.di_pair_job_items(1 << 20, 4096, 128) == -2
    p = ctypes.c_void_p(16)
    assert lib.di_pair_signal(None, 0, None) == -1
    assert lib.di_pair_signal(p, -1, None) == -1
    assert lib.di_pair_stream(_lib.DI_BF16, p, 3, 3, 128, p, None, 20.0, None) == -1   # empty range
    assert lib.di_pair_stream(_lib.DI_BF16, p, 0, 4, 128, p, None, 0.0, None) == -1    # no patience
    assert lib.di_pair_stream(5, p, 0, 4, 128, p, None, 20.0, None) == -1             # dtype
    bad = _lib.DiPairLaunch(0, 0, 17, 1)
    assert lib.di_pair_stream(_lib.DI_BF16, p, 0, 4, 128, p, ctypes.byref(bad), 20.0, None) == -1
    assert lib.di_pair_help(_lib.DI_BF16, p, 4, 3, 128, p, None, -1, None) == -1
    assert lib.di_pair_help(_lib.DI_F32, None, 0, 3, 128, p, None, -1, None) == -1
    assert lib.di_pair_help(_lib.DI_F32, p, 0, 3, 128, p, ctypes.byref(bad), -1, None) == -1


def test_stream_helpers_host_contract():
    """ABI 8's stream helpers refuse bad arguments before touching the device."""
    lib = _lib.load()
    assert lib.di_stream_create_dedicated(None) == -1
    assert lib.di_stream_destroy(None) == -1
    out = ctypes.c_int32(7)
    p, q = ctypes.c_void_p(16), ctypes.c_void_p(32)
    assert lib.di_streams_concurrent(p, q, None, 100.0, ctypes.byref(out)) == -1       # no work buffer
    assert lib.di_streams_concurrent(p, q, p, 0.0, ctypes.byref(out)) == -1            # no patience
    assert lib.di_streams_concurrent(p, q, p, 20000.0, ctypes.byref(out)) == -1        # too long
    assert lib.di_streams_concurrent(p, p, p, 100.0, ctypes.byref(out)) == -1          # one stream
    assert lib.di_streams_concurrent(p, q, p, 100.0, None) == -1
    assert out.value == 7


def _declared_struct_fields(name):
    src = open(os.path.join(ROOT, "include", "deepinteract_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    for m in re.finditer(r"typedef struct \{(.*?)\}\s*(\w+);", src, flags=re.S):
        if m.group(2) == name:
            fields = []
            for decl in m.group(1).split(";"):
                decl = decl.strip()
                if decl:
                    fields += [f.strip().lstrip("*") for f in decl.split(None, 1)[1].split(",")] \
                        if "," in decl else [decl.split()[-1].lstrip("*")]
            return fields
    raise KeyError(name)


def test_ctypes_struct_fields_match_header():
    for cls, name in ((_lib.DiGraph, "di_graph"), (_lib.DiPairDesc, "di_pair_desc"), (_lib.DiGeoArgs, "di_geo_args"),
                      (_lib.DiPairJob, "di_pair_job")):
        assert [f for f, _ in cls._fields_] == _declared_struct_fields(name), name


def _declared_arg_counts():
    """function name -> number of parameters, parsed from include/deepinteract_amd.h."""
    src = open(os.path.join(ROOT, "include", "deepinteract_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|int32_t|int64_t)\s+(di_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", src):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return out


def test_ctypes_signatures_match_header():
    """Every entry point the header declares is bound in _lib._SIGS with the header's argument
    count (a stale ctypes signature would pass garbage through the boundary)."""
    decl = _declared_arg_counts()
    assert set(decl) == set(declared_symbols())
    assert set(decl) == set(_lib._SIGS), set(decl) ^ set(_lib._SIGS)
    for name, n in decl.items():
        assert len(_lib._SIGS[name][0]) == n, (name, len(_lib._SIGS[name][0]), n)


def test_integration_stub_matches_header():
    """INTEGRATION.md's raw-C (ctypes) stub passes as many arguments as the header declares."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    decl = _declared_arg_counts()
    calls = re.findall(r"\blib\.(di_[a-z0-9_]+)\(", text)
    assert calls, "INTEGRATION.md has no ctypes stub calls"
    for m in re.finditer(r"\blib\.(di_[a-z0-9_]+)\(", text):
        depth, i = 1, m.end()
        while depth:
            depth += {"(": 1, ")": -1}.get(text[i], 0)
            i += 1
        body = text[m.end():i - 1]
        # count top-level commas
        n, d = (1 if body.strip() else 0), 0
        for ch in body:
            d += {"(": 1, "[": 1, ")": -1, "]": -1}.get(ch, 0)
            n += ch == "," and d == 0
        assert n == decl[m.group(1)], (m.group(1), n, decl[m.group(1)])


def test_build_stamp_is_path_independent():
    """The in-tree library counts as built when the tree is copied elsewhere (the GPU box runs the
    snapshot at another path, without building): the stamp holds no absolute repo path and the
    library built here is current."""
    root = os.path.dirname(build.HERE)
    assert root not in build._stamp()
    assert build.up_to_date()
