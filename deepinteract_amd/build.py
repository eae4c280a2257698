"""Build the in-tree HIP shared library for gfx950: deepinteract_amd/lib/libdeepinteract_amd.so.

Plain ``hipcc -shared -fPIC --offload-arch=gfx950`` over every csrc/*.hip file (one
translation unit each, compiled in parallel, then linked). The .so lives in-tree so it
travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libdeepinteract_amd.so")
ARCH = os.environ.get("DI_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          f"-I{os.path.join(os.path.dirname(HERE), 'include')}"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _deps():
    return _sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + \
        [os.path.join(os.path.dirname(HERE), "include", "deepinteract_amd.h"), os.path.abspath(__file__)]


def _stamp(defines=(), link_flags=()) -> str:
    """What a build of the library depends on (written next to every built library): compiler,
    flags, arch, the -D defines of a variant, the link flags and a hash of every source / header /
    this file's contents. Repo-relative, so a tree copied to another path (the GPU box's snapshot,
    whose extraction need not keep mtimes) still matches the library built here."""
    root = os.path.dirname(HERE)
    h = hashlib.sha256()
    for p in _deps():
        h.update(os.path.relpath(p, root).encode())
        with open(p, "rb") as fh:
            h.update(fh.read())
    cflags = [f.replace(root, "<repo>") for f in CFLAGS]
    return json.dumps({"hipcc": HIPCC, "cflags": cflags, "arch": ARCH, "defines": list(defines),
                       "link": list(link_flags), "sources": h.hexdigest()}, sort_keys=True)


def _fresh(lib_path: str, defines=(), link_flags=()) -> bool:
    """lib_path exists and was built from the same sources with the same compiler, flags and
    defines (its .stamp file)."""
    if not os.path.exists(lib_path):
        return False
    try:
        with open(lib_path + ".stamp") as fh:
            if fh.read() != _stamp(defines, link_flags):
                return False
    except OSError:
        return False
    return True


def up_to_date() -> bool:
    return _fresh(LIB)


# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of the C ABI (argument validation,
# descriptor / size arithmetic, launch-shape selection): every -fsanitize flag applies to the host
# compilation only (-Xarch_host); device code is unchanged and GPU sanitizers are not used. Loaded in
# a child process with the shared ASan runtime preloaded (tests/test_host_sanitizers.py).
SAN_FLAGS = ["-O1", "-g", "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer"]
SAN_LIB = os.path.join(LIBDIR, "asan", "libdeepinteract_amd.so")


def asan_runtime() -> str:
    """The shared ASan runtime of the ROCm LLVM the library is built with."""
    cands = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not cands:
        raise RuntimeError("libclang_rt.asan-x86_64.so not found under /opt/rocm/lib/llvm")
    return cands[-1]


SAN_LINK = ["-fsanitize=address", "-fsanitize=undefined", "-shared-libsan"]


def build_host_sanitized(force: bool = False) -> str:
    return build(force=force, defines=SAN_FLAGS, out=SAN_LIB, link_flags=SAN_LINK)


def build(force: bool = False, verbose: bool = True, defines=(), out: str | None = None, link_flags=()) -> str:
    """Build the library. ``defines``/``out`` build a tuning variant (extra -D defines, or raw
    compiler flags when an entry starts with '-') into its
    own directory, loaded with bench.py --lib <path> (launch-shape knobs compared in one GPU session)."""
    lib_path = out or LIB
    if not force and _fresh(lib_path, defines, link_flags):
        return lib_path
    objdir = os.path.join(os.path.dirname(lib_path), "obj")
    os.makedirs(objdir, exist_ok=True)
    objs = []

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        cmd = [HIPCC, *CFLAGS, *[d if d.startswith("-") else f"-D{d}" for d in defines], "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, len(_sources()))) as ex:
        objs = list(ex.map(compile_one, _sources()))
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", *link_flags, "-o", lib_path, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    with open(lib_path + ".stamp", "w") as fh:
        fh.write(_stamp(defines, link_flags))
    if verbose:
        print(f"built {lib_path}", file=sys.stderr)
    return lib_path


def build_variant(name: str, defines) -> str:
    return build(defines=defines, out=os.path.join(LIBDIR, "variants", name, "libdeepinteract_amd.so"))


if __name__ == "__main__":
    build(force="--force" in sys.argv)
