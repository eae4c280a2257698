"""Timing-diagnostic builds of the library from PATCHED COPIES of csrc/ (never -D knobs in the
product sources): each diagnostic is a list of exact text substitutions applied to a copy of
deepinteract_amd/csrc + include/, built into deepinteract_amd/lib/variants/diag_<name>/ and loaded
with bench.py --lib. Every diagnostic computes WRONG results on purpose (timing only).

usage: python tools/diag/patch_build.py nosilu nosync w0 ...
"""
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from deepinteract_amd import build  # noqa: E402

DIAGS = {
    # the edge layers' SiLU epilogues as a plain multiply (no transcendentals): how much of the step a
    # faster GeoT converts into throughput
    "nosilu": [("mfma32.h", "for (int k = 0; k < 16; ++k) v[k] = silu2<true>(v[k]);",
                "for (int k = 0; k < 16; ++k) v[k] = v[k] * 0.5f;", 1)],
    # the double-buffered weight stages switch without waiting for their LDS-DMA or a barrier
    "nosync": [("common.h", """    if constexpr (DBUF) {
      lds_dma_wait();
      __syncthreads();
      cur ^= 1;""", """    if constexpr (DBUF) {
      cur ^= 1;""", 1)],
    # every bf16 edge-layer weight stage DMA'd from the blob's first blocks: the weight stream always
    # hits L2 (same bytes, same instruction count; wrong weights)
    "w0": [("geot_kernels.hip", "    pipe.issue(W + EL_ORDER[si] * BLK, EL_SIZE[si], vo >= 0 ? V + vo : nullptr, 128);\n  }\n  __device__ const u16* next() {",
            "    pipe.issue(W, EL_SIZE[si], vo >= 0 ? V : nullptr, 128);\n  }\n  __device__ const u16* next() {", 1)],
}


def build_diag(name):
    tmp = tempfile.mkdtemp(prefix=f"di_diag_{name}_")
    try:
        src = os.path.join(tmp, "deepinteract_amd", "csrc")
        shutil.copytree(build.CSRC, src)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
        for fname, old, new, count in DIAGS[name]:
            p = os.path.join(src, fname)
            text = open(p).read()
            if text.count(old) != count:
                raise SystemExit(f"diag {name}: pattern found {text.count(old)}x in {fname}, expected {count}")
            open(p, "w").write(text.replace(old, new))
        out = os.path.join(build.LIBDIR, "variants", f"diag_{name}", "libdeepinteract_amd.so")
        saved = build.CSRC, build.CFLAGS
        build.CSRC = src
        build.CFLAGS = [f for f in build.CFLAGS if not f.startswith("-I")] + [f"-I{os.path.join(tmp, 'include')}"]
        try:
            return build.build(force=True, defines=[f"DI_TIMING_DIAG_{name.upper()}=1"], out=out)
        finally:
            build.CSRC, build.CFLAGS = saved
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(DIAGS):
        print(build_diag(n))
