"""A/B builds against a committed tree: build the library from csrc/ + include/ as they are at a git
revision into deepinteract_amd/lib/variants/rev_<name>/ (bench.py --lib / tools/diag/* --lib).

usage: python tools/diag/build_rev.py <name> [<revision>]   (revision: default HEAD)
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from deepinteract_amd import build  # noqa: E402


def build_rev(name, rev="HEAD"):
    tmp = tempfile.mkdtemp(prefix=f"di_rev_{name}_")
    try:
        src = os.path.join(tmp, "deepinteract_amd", "csrc")
        inc = os.path.join(tmp, "include")
        os.makedirs(src)
        os.makedirs(inc)
        for d, out in (("deepinteract_amd/csrc", src), ("include", inc)):
            names = subprocess.check_output(["git", "-C", ROOT, "ls-tree", "--name-only", rev, d + "/"], text=True).split()
            for path in names:
                data = subprocess.check_output(["git", "-C", ROOT, "show", f"{rev}:{path}"])
                with open(os.path.join(out, os.path.basename(path)), "wb") as fh:
                    fh.write(data)
        out = os.path.join(build.LIBDIR, "variants", f"rev_{name}", "libdeepinteract_amd.so")
        saved = build.CSRC, build.CFLAGS
        build.CSRC = src
        build.CFLAGS = [f for f in build.CFLAGS if not f.startswith("-I")] + [f"-I{inc}"]
        try:
            return build.build(force=True, defines=[f"DI_REV_{name.upper()}=1"], out=out)
        finally:
            build.CSRC, build.CFLAGS = saved
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    print(build_rev(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "HEAD"))
