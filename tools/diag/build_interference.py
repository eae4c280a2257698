"""Diagnostic builds (NOT shipped; WRONG RESULTS by design) that locate the interference between
GeoT and the pair-tensor store stream. Patched sources go to lib/variants/<name>/src.
  nostore  the grouped edge kernel's F_out / Fn_out row stores folded onto 16 rows (L2-resident):
           is the edge layer slowed by its own 164 MB of scattered 32-B row-piece writes?
  pairl2   the bounded row-streaming pair kernel's stores folded onto a 64-KiB window per plane
           (same instructions through the CU's memory pipeline, no HBM write stream): is the
           slowdown CU-local (issue / vector-memory queue) or in the memory system?
usage: python tools/diag/build_nostore.py [nostore|pairl2]   then   bench.py --lib lib/variants/<name>/..."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from deepinteract_amd import build  # noqa: E402

NAME = sys.argv[1] if len(sys.argv) > 1 else "nostore"
out = os.path.join(build.LIBDIR, "variants", NAME)
src = os.path.join(out, "src")
shutil.rmtree(src, ignore_errors=True)
shutil.copytree(build.CSRC, src)
for f in os.listdir(src):
    fp = os.path.join(src, f)
    t = open(fp).read().replace('"../../include/deepinteract_amd.h"', '"deepinteract_amd.h"')
    open(fp, "w").write(t)
p = os.path.join(src, "geot_kernels.hip" if NAME == "nostore" else "pair_tensor.hip")
s = open(p).read()
for old in () if NAME != "nostore" else ("store_row(e1[q], reinterpret_cast<u16*>(a.f_out) + (int64_t)rw[q].e * HID, g)",
            "store_row(fn, reinterpret_cast<u16*>(a.fn_out) + (int64_t)rw[q].e * HID, g)"):
    assert old in s, "k_edge_lean stores changed; update the patch"
    s = s.replace(old, old.replace("(int64_t)rw[q].e * HID", "(int64_t)(rw[q].e & 15) * HID"))
if NAME == "pairl2":
    old = "const int soff = (int)(i * pitch);"
    assert old in s, "k_pair_rows changed; update the patch"
    s = s.replace(old, "const int soff = (int)(i * pitch) & 0xffff;")
open(p, "w").write(s)
shutil.copy(os.path.join(ROOT, "include", "deepinteract_amd.h"), src)
old_csrc = build.CSRC
build.CSRC = src
try:
    print(build.build(out=os.path.join(out, "libdeepinteract_amd.so")))
finally:
    build.CSRC = old_csrc
