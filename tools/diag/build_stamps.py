"""Diagnostic build (NOT shipped): the edge kernels with s_memtime stamps around every weight-stage
switch. Lane 0 of every wave of the first 64 blocks records, for its first tile, the cycle it
reaches EdgeStages::next() and the cycle it leaves it (after the stage's wait) into a debug buffer
no kernel code reads (MI355X_MICROARCH.md DVFS item 6: stamps never feed an output). The patched
sources go to lib/variants/stamps/src; the product sources are untouched.
usage: python tools/diag/build_stamps.py [extra -D defines]"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from deepinteract_amd import build  # noqa: E402

name = "stamps" + ("_" + "_".join(d.split("=")[0].lower() for d in sys.argv[1:]) if sys.argv[1:] else "")
out = os.path.join(build.LIBDIR, "variants", name)
src = os.path.join(out, "src")
shutil.rmtree(src, ignore_errors=True)
shutil.copytree(build.CSRC, src)
for f in os.listdir(src):
    fp = os.path.join(src, f)
    t = open(fp).read().replace('"../../include/deepinteract_amd.h"', '"deepinteract_amd.h"')
    open(fp, "w").write(t)
p = os.path.join(src, "geot_kernels.hip")
s = open(p).read()
s = s.replace("namespace di {\n\nstruct EmbedArgs", """namespace di {
__device__ unsigned long long* g_stamps = nullptr;  // [64 blocks][8 waves][64 stages][3]
__device__ __forceinline__ void stamp(int slot) {
  unsigned long long* b = g_stamps;
  if (b == nullptr || blockIdx.x >= 64 || (threadIdx.x & 63) != 0 || slot >= 192) return;
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  b[((size_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * 192 + slot] = t;
}

struct EmbedArgs""", 1)
s = s.replace("""  __device__ const T* next() {
    const int i = gi++;""", """  __device__ const T* next() {
    const int i = gi++;
    if (i < 64) stamp(3 * i);
    struct Leave { int i; __device__ ~Leave() { if (i < 64) stamp(3 * i + 2); } } leave_{i};""", 1)
s = s.replace("      if (i + 2 < total) issue(i + 2);", "      if (i < 64) stamp(3 * i + 1);\n      if (i + 2 < total) issue(i + 2);", 1)
s = s.replace("      if (i + 1 < total) issue(i + 1);", "      if (i < 64) stamp(3 * i + 1);\n      if (i + 1 < total) issue(i + 1);", 1)
s = s.replace('extern "C" int di_abi_version(void) { return DI_ABI_VERSION; }', '''extern "C" int di_abi_version(void) { return DI_ABI_VERSION; }
extern "C" int di_diag_stamps(void* buf) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf)); }''', 1)
open(p, "w").write(s)
old_csrc = build.CSRC
build.CSRC = src
try:
    print(build.build(defines=sys.argv[1:], out=os.path.join(out, "libdeepinteract_amd.so")))
finally:
    build.CSRC = old_csrc
