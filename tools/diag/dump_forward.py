"""Bit-exactness of an A/B build (tools/diag/patch_build.py variants marked correct) against the
product library: one bf16 GeoT forward over a C3 micro-batch (8 complexes of 1000 x 1000, k = 20),
its node and edge outputs saved for tools/diag/dump_forward.py --compare. One library per process.

usage (GPU box): python tools/diag/dump_forward.py [--lib variant.so] --out a.pt
                 python tools/diag/dump_forward.py --compare a.pt b.pt
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--compare", nargs=2, default=None)
    args = ap.parse_args()
    if args.compare:
        a, b = (torch.load(p, weights_only=True) for p in args.compare)
        same = {k: bool(torch.equal(a[k], b[k])) for k in a}
        print({"bit_identical": same})
        sys.exit(0 if all(same.values()) else 1)
    from deepinteract_amd import _lib, synth
    if args.lib:
        _lib.load_variant(args.lib)
    from deepinteract_amd.builder import build_graph_batch
    from deepinteract_amd.engine import GeoTEngine
    from deepinteract_amd.weights import seeded_state_dict
    dev = torch.device("cuda")
    eng = GeoTEngine(seeded_state_dict(0, with_head=False), "bf16", device=dev)
    chains = [c for j in range(8) for c in synth.synthetic_complex(300 + j, 1000, 1000)]
    gb = build_graph_batch(chains, k=20, nbr_seeds=list(range(1, 17)), device=dev)
    node, edge = eng.forward(gb)
    torch.cuda.synchronize()
    torch.save({"node": node.view(torch.int16).cpu(), "edge": edge.view(torch.int16).cpu(),
                "hT": eng.last_hT.view(torch.int16).cpu()}, args.out)


if __name__ == "__main__":
    main()
