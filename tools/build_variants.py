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
    "prio2": ["DI_GEOT_PRIO=2"],
    "prio3": ["DI_GEOT_PRIO=3"],
    "persist": ["DI_EDGE_PERSIST=1"],
    # grouped/lean edge layer (bench --edge-kernel 1): waves per block, waves per SIMD, VGPR cap / 2
    "lean4": ["DI_LEAN_NW=4", "DI_LEAN_WPE=2", "DI_LEAN_VGPR=120"],
    "lean6": ["DI_LEAN_NW=6", "DI_LEAN_WPE=3", "DI_LEAN_VGPR=80"],
    "lean8": ["DI_LEAN_NW=8", "DI_LEAN_WPE=4", "DI_LEAN_VGPR=64"],
    "lean12": ["DI_LEAN_NW=12", "DI_LEAN_WPE=3", "DI_LEAN_VGPR=80"],
    "lean4d6": ["DI_LEAN_NW=4", "DI_LEAN_WPE=2", "DI_LEAN_VGPR=120", "DI_MMA_DEPTH=6"],
    "lean4d10": ["DI_LEAN_NW=4", "DI_LEAN_WPE=2", "DI_LEAN_VGPR=120", "DI_MMA_DEPTH=10"],
    "lean12d6": ["DI_LEAN_NW=12", "DI_LEAN_WPE=3", "DI_LEAN_VGPR=80", "DI_MMA_DEPTH=6"],
    "lean8d5": ["DI_LEAN_NW=8", "DI_LEAN_WPE=4", "DI_LEAN_VGPR=64", "DI_MMA_DEPTH=5"],
    "base_ring8": ["DI_MMA_ORDER=4", "DI_MMA_DEPTH=8"],
    "lean4s3": ["DI_LEAN_NW=4", "DI_LEAN_WPE=3", "DI_LEAN_VGPR=80", "DI_LEAN_DBUF=0", "DI_MMA_DEPTH=6"],
    "lean4s4": ["DI_LEAN_NW=4", "DI_LEAN_WPE=4", "DI_LEAN_VGPR=64", "DI_LEAN_DBUF=0", "DI_MMA_DEPTH=5"],
    "lean8d5v60": ["DI_LEAN_NW=8", "DI_LEAN_WPE=4", "DI_LEAN_VGPR=60", "DI_MMA_DEPTH=5"],
    "lean4g2": ["DI_LEAN_NW=4", "DI_LEAN_WPE=2", "DI_LEAN_VGPR=120", "DI_LEAN_G=2"],
    "lean4g2d6": ["DI_LEAN_NW=4", "DI_LEAN_WPE=2", "DI_LEAN_VGPR=120", "DI_LEAN_G=2", "DI_MMA_DEPTH=6"],
    "lean4g2ns": ["DI_LEAN_NW=4", "DI_LEAN_WPE=2", "DI_LEAN_VGPR=120", "DI_LEAN_G=2", "DI_LEAN_SHARE=0"],
    "lean4g2d4": ["DI_LEAN_NW=4", "DI_LEAN_WPE=2", "DI_LEAN_VGPR=120", "DI_LEAN_G=2", "DI_MMA_DEPTH=4"],
    "pst_plain": ["DI_PAIR_STORE_BESIDE=0"],
    "pst_ntsc0": ["DI_PAIR_STORE_BESIDE=3"],
    "edge_nt": ["DI_EDGE_ROW_NT=1"],
    "f16res": ["DI_LEAN_F16RES=1"],
    "init_d2": ["DI_INIT_DBUF=1", "DI_INIT_WPE=2"],
    "init_s4": ["DI_INIT_DBUF=0", "DI_INIT_WPE=4"],
    "g1s4": ["DI_LEAN_G=1", "DI_LEAN_NW=4", "DI_LEAN_WPE=4", "DI_LEAN_VGPR=64", "DI_LEAN_DBUF=0", "DI_MMA_DEPTH=5"],
    "g1s3": ["DI_LEAN_G=1", "DI_LEAN_NW=4", "DI_LEAN_WPE=3", "DI_LEAN_VGPR=80", "DI_LEAN_DBUF=0", "DI_MMA_DEPTH=6"],
    "g1s2": ["DI_LEAN_G=1"],
    "gc_d3": ["DI_MMA_DEPTH=3"],
    "gc_d6": ["DI_MMA_DEPTH=6"],
    "gc_nofence": ["DI_LEAN_FENCE=0"],
    "gc_holdf": ["DI_LEAN_HOLD_F=1"],
    "nt_if4": ["DI_PAIR_INFLIGHT=4"],
    "nt_if6": ["DI_PAIR_INFLIGHT=6"],
    "nt_if2": ["DI_PAIR_INFLIGHT=2"],
    "inflight1": ["DI_PAIR_INFLIGHT=1"],
    "inflight2": ["DI_PAIR_INFLIGHT=2"],
    "inflight3": ["DI_PAIR_INFLIGHT=3"],
    "inflight4": ["DI_PAIR_INFLIGHT=4"],
    "inflight6": ["DI_PAIR_INFLIGHT=6"],
    "inflight8": ["DI_PAIR_INFLIGHT=8"],
    "inflight16": ["DI_PAIR_INFLIGHT=16"],
    "lean8g2": ["DI_LEAN_NW=8", "DI_LEAN_WPE=2", "DI_LEAN_VGPR=120", "DI_LEAN_G=2", "DI_MMA_DEPTH=6"],
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    with cf.ThreadPoolExecutor(2) as ex:
        for p in ex.map(lambda n: build.build_variant(n, VARIANTS[n]), names):
            print(p)
