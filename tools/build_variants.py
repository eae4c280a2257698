"""Build kernel-tuning variants of the library (lib/variants/<name>/), compared on the GPU in
one session with bench.py --lib <path> (tools/variants.sh)."""
import concurrent.futures as cf
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deepinteract_amd import build

VARIANTS = {
    # the product library's only compile-time knob (csrc/geot_kernels.hip DI_NODE_NW): k_node_layer in
    # 2-wave blocks; every launch site takes its shape from NodeGeo, and tests/test_gpu_node_aggr.py
    # runs against this build (DI_TEST_VARIANT) to keep the non-default value tested
    "node2": ["DI_NODE_NW=2"],
    # round 3: fp32 SiLU as libm expf + IEEE division (the round-2 default)
    "f32exact": ["DI_F32_FAST_SILU=0"],
    # round 4: the bf16 edge layers on the round-3 16x16x32 kernel (k_edge_lean, 16-row blobs)
    "lean16": ["DI_EDGE_X32=0"],
    # round 4: the bf16 InitEdge kernels on 16x16x32 (k_init_edge / k_init_edge_res, 16-row blob)
    "init16": ["DI_INIT_X32=0"],
    # round 4: pair stores beside GeoT with the row-boundary partial lines as plain stores
    "pairedge": ["DI_PAIR_EDGE_PLAIN=1"],
    # round 4: pair-store waves at raised issue priority beside GeoT
    "pprio1": ["DI_PAIR_PRIO=1"],
    "pprio3": ["DI_PAIR_PRIO=3"],
    # round 4: pair stores beside GeoT as sc1 / sc0 sc1 / sc1 nt (dropped from L2) instead of nt
    "cpol0": ["DI_PAIR_CPOL=0"],
    "cpol1": ["DI_PAIR_CPOL=1"],
    "cpol16": ["DI_PAIR_CPOL=16"],
    "cpol17": ["DI_PAIR_CPOL=17"],
    "cpol18": ["DI_PAIR_CPOL=18"],
    # round 4: chain-1 pair planes as contiguous whole-line runs (nt / sc1 beside GeoT)
    "c1run": ["DI_PAIR_C1RUN=1"],
    "c1run16": ["DI_PAIR_C1RUN=1", "DI_PAIR_C1CPOL=16"],
    "c1runb2": ["DI_PAIR_C1RUN=1", "DI_PAIR_C1BOUND=2"],
    "c1runb3": ["DI_PAIR_C1RUN=1", "DI_PAIR_C1BOUND=3"],
    "c1runp3": ["DI_PAIR_C1RUN=1", "DI_PAIR_PRIO=3"],
    # round 4: pair stores in flight per wave beside GeoT (default 3)
    "infl4": ["DI_PAIR_INFLIGHT=4"],
    "infl5": ["DI_PAIR_INFLIGHT=5"],
    # round 4: both InitEdge and the edge layers on 16x16x32 (the round-3 kernels)
    "x16": ["DI_EDGE_X32=0", "DI_INIT_X32=0"],
    # round 4: k_edge_x32 epilogue density (VALU per MFMA) and fragment prefetch depth
    "nv4": ["DI_PIPE32_NV=4"],
    "nv12": ["DI_PIPE32_NV=12"],
    "depth6": ["DI_MMA_DEPTH=6"],
    # round 4: epi(ob - 1)'s VALU after 2 of block ob's MFMAs; static s_setprio 1 for odd edge blocks
    "lead2": ["DI_PIPE32_LEAD=2"],
    "eprio": ["DI_EDGE_PRIO=1"],
    # round 4: k_edge_x32's row re-reads / K,Q gathers issued after the stage barriers
    "rowld": ["DI_X32_ROWLD=1"],
    # round 4: each linear's block-3 epilogue under the next linear's first MFMAs (k_edge_x32 chain)
    "defer": ["DI_X32_DEFER=1"],
    # round 4: the edge row's lines touched one stage ahead of each re-read (L2 prefetch)
    "pfetch": ["DI_X32_PREFETCH=1"],
    # timing diagnostics (wrong results; bench only): no SiLU transcendentals / no stage waits
    "nosilu": ["DI_DIAG_NOSILU=1"],
    "nosync": ["DI_DIAG_NOSYNC=1"],
    "reread0": ["DI_DIAG_REREAD0=1"],
}
# New experiments add their -D knob to csrc (defaulting to the shipped value) and an entry here;
# round 2's knobs (edge ring / persistent tiles / XCD tile order / DMA pumping / f16 ResBlocks / pair
# pacing, ...) and round 3's scalar-VALU build were measured, recorded in DESIGN.md §8 and removed from the sources.

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    with cf.ThreadPoolExecutor(2) as ex:
        for p in ex.map(lambda n: build.build_variant(n, VARIANTS[n]), names):
            print(p)
