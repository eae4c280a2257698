"""Build kernel-tuning variants of the library (lib/variants/<name>/), compared on the GPU in
one session with bench.py --lib <path> (tools/variants.sh)."""
import concurrent.futures as cf
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deepinteract_amd import build

VARIANTS = {
    # launch-shape / schedule knobs only: every variant computes the same results
    "base": [],
    "order1": ["DI_MMA_ORDER=1"],
    "order2": ["DI_MMA_ORDER=2"],
    "noslp": ["-fno-slp-vectorize"],
    "xcd": ["DI_XCD_TILES=1"],
    "prio1": ["DI_GEOT_PRIO=1"],
    "persist": ["DI_EDGE_PERSIST=1"],
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    with cf.ThreadPoolExecutor(2) as ex:
        for p in ex.map(lambda n: build.build_variant(n, VARIANTS[n]), names):
            print(p)
