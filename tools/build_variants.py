"""Build kernel-tuning variants of the library (lib/variants/<name>/), compared on the GPU in
one session with bench.py --lib <path> (tools/variants.sh)."""
import concurrent.futures as cf
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deepinteract_amd import build

VARIANTS = {
    # the product library's compile-time knobs, each kept tested by a -m gpu test against its variant:
    # k_node_layer in 2-wave blocks (csrc/geot_kernels.hip DI_NODE_NW; every launch site takes its shape
    # from NodeGeo; tests/test_gpu_variants.py, tests/test_gpu_node_aggr.py via DI_TEST_VARIANT)
    "node2": ["DI_NODE_NW=2"],
    # fp32 SiLU as libm expf + IEEE division (csrc/common.h DI_F32_FAST_SILU; the round-2 default)
    "f32exact": ["DI_F32_FAST_SILU=0"],
}
# Rejected experiments are recorded in DESIGN.md §8 and removed from the sources; timing diagnostics
# that need patched kernels are built from patched source copies by tools/diag/ (never -D knobs in csrc).

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    with cf.ThreadPoolExecutor(2) as ex:
        for p in ex.map(lambda n: build.build_variant(n, VARIANTS[n]), names):
            print(p)
