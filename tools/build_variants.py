"""Build kernel-tuning variants of the library (lib/variants/<name>/), compared on the GPU in
one session with DI_LIB=<path> (tools/variants.sh)."""
import concurrent.futures as cf
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deepinteract_amd import build

VARIANTS = {
    "base": [],
    "order1": ["DI_MMA_ORDER=1"],
    "order2": ["DI_MMA_ORDER=2"],
    "order3": ["DI_MMA_ORDER=3"],
    "nobar": ["DI_X_NOBAR"],
    "nosilu": ["DI_X_NOSILU"],
    "halfsilu": ["DI_X_HALFSILU"],
    "nodma": ["DI_X_NODMA"],
    "nodma_nobar": ["DI_X_NODMA", "DI_X_NOBAR"],
    "nodma_nosilu": ["DI_X_NODMA", "DI_X_NOSILU"],
    "nodma_nobar_nosilu": ["DI_X_NODMA", "DI_X_NOBAR", "DI_X_NOSILU"],
    "strip_noldsa": ["DI_X_NODMA", "DI_X_NOBAR", "DI_X_NOSILU", "DI_X_NOLDSA"],
    "noldsa": ["DI_X_NOLDSA"],
    "nopersist": ["DI_EDGE_PERSIST=0"],
    "nopp": ["DI_EDGE_PP=0"],
    "pp_persist": ["DI_EDGE_PERSIST=1"],
    "pp_prio": ["DI_X_PRIO=1"],
    "pp_nomid": ["DI_X_NOMID"],
    "stagger40": ["DI_X_STAGGER=40"],
    "stagger120": ["DI_X_STAGGER=120"],
    "nw8": ["DI_GEO_NW=8"],
    "nw8_order3": ["DI_GEO_NW=8", "DI_MMA_ORDER=3"],
    "noslp": ["-fno-slp-vectorize"],
    "prow_strided": ["DI_PAIR_ROWS_STRIDED"],
    "prow_plain": ["DI_PAIR_STORE=0"],
    "prow_legacy": ["DI_PAIR_LEGACY"],
    "prow_w1": ["DI_PAIR_ROW_WAVES=1"],
    "prow_w8": ["DI_PAIR_ROW_WAVES=8"],
    "prow_w16": ["DI_PAIR_ROW_WAVES=16"],
    "pump1": ["DI_DMA_PUMP=1"],
    "pump2": ["DI_DMA_PUMP=2"],
    "pump4": ["DI_DMA_PUMP=4"],
    "prow_w2": ["DI_PAIR_ROW_WAVES=2"],
    "nw8_nobar": ["DI_GEO_NW=8", "DI_X_NOBAR"],
    "nw8_nodma": ["DI_GEO_NW=8", "DI_X_NODMA"],
    "nw8_nodma_nobar": ["DI_GEO_NW=8", "DI_X_NODMA", "DI_X_NOBAR"],
    "pair_sc1": ["DI_PAIR_STORE=16"],
    "pair_sc1nt": ["DI_PAIR_STORE=18"],
    "xcd": ["DI_XCD_TILES=1"],
    "prio1": ["DI_GEOT_PRIO=1"],
    "prio3": ["DI_GEOT_PRIO=3"],
    "persist_prio2": ["DI_EDGE_PERSIST=1", "DI_GEOT_PRIO=2"],
    "vgpr128": ["DI_EDGE_NUM_VGPR=128"],
    "vgpr124": ["DI_EDGE_NUM_VGPR=124"],
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    with cf.ThreadPoolExecutor(2) as ex:
        for p in ex.map(lambda n: build.build_variant(n, VARIANTS[n]), names):
            print(p)
