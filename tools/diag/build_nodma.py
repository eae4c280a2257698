"""Diagnostic build (NOT shipped; WRONG RESULTS by design): the edge kernels with the weight
stream switched off after the first two stages — every later stage reads the stale weights of
slot i&1, with no LDS-DMA and no stage barrier. Times the row-on-lane MFMA/VALU chain alone
(the compute-only floor of k_edge_layer). Patched sources go to
lib/variants/nodma/src; the product sources are untouched.
usage: python tools/diag/build_nodma.py   then   bench.py --lib lib/variants/nodma/... --overlap 0"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from deepinteract_amd import build  # noqa: E402

out = os.path.join(build.LIBDIR, "variants", "nodma")
src = os.path.join(out, "src")
shutil.rmtree(src, ignore_errors=True)
shutil.copytree(build.CSRC, src)
for f in os.listdir(src):
    fp = os.path.join(src, f)
    t = open(fp).read().replace('"../../include/deepinteract_amd.h"', '"deepinteract_amd.h"')
    open(fp, "w").write(t)
p = os.path.join(src, "geot_kernels.hip")
s = open(p).read()
old = """    } else {
      const T* w = pipe.next();
      if (i + 1 < total) issue(i + 1);"""
assert old in s, "EdgeStages::next() changed; update the patch"
s = s.replace(old, """    } else {
      if (i >= 2) {
        vcur = pipe.slot_v(i & 1);
        return pipe.slot_w(i & 1);
      }
      const T* w = pipe.next();
      if (i + 1 < total) issue(i + 1);""", 1)
open(p, "w").write(s)
old_csrc = build.CSRC
build.CSRC = src
try:
    print(build.build(out=os.path.join(out, "libdeepinteract_amd.so")))
finally:
    build.CSRC = old_csrc
