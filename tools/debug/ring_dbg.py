"""Debug: edge-layer outputs of the product library vs a variant library on the same inputs, per row
(wave slot within a 256-row tile) and feature. usage: python tools/debug/ring_dbg.py <variant.so>"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(out, lib=None):
    import torch
    from deepinteract_amd import _lib
    if lib:
        _lib.load_variant(lib)
    from gpu_common import chain_item, load_case
    from deepinteract_amd.engine import GeoTEngine
    from deepinteract_amd.graph import GraphBatch
    from deepinteract_amd.weights import seeded_state_dict
    z = load_case(sys.argv[2] if len(sys.argv) > 2 else "tiny")
    gb = GraphBatch.from_arrays([chain_item(z, "g1"), chain_item(z, "g2")], "cuda")
    eng = GeoTEngine(seeded_state_dict(0), "bf16")
    h, e = eng.forward(gb)
    torch.cuda.synchronize()
    np.savez(out, h=h.float().cpu().numpy(), e=e.float().cpu().numpy(), geo_ref=gb.geo_ref)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        run(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != "-" else None)
        sys.exit(0)
    O = os.path.join(ROOT, "gpurun_out")
    case = sys.argv[2] if len(sys.argv) > 2 else "tiny"
    for tag, lib in (("prod", "-"), ("var", sys.argv[1])):
        subprocess.run([sys.executable, __file__, "--child", f"{O}/ringdbg_{tag}.npz", lib, case][:5] if False else
                       [sys.executable, __file__, "--child", f"{O}/ringdbg_{tag}.npz", lib], check=True)
    a, b = np.load(f"{O}/ringdbg_prod.npz"), np.load(f"{O}/ringdbg_var.npz")
    print("geo_ref", a["geo_ref"])
    for k in ("h", "e"):
        d = np.abs(a[k] - b[k])
        print(k, "max diff", d.max(), "rel", d.max() / np.abs(b[k]).max())
        rows = np.where(d.max(1) > 1e-2 * np.abs(b[k]).max())[0]
        print("  bad rows", len(rows), "of", len(d))
        if len(rows):
            print("  first", rows[:20], "wave slots", np.bincount((rows % 256) // 32, minlength=8), "tiles",
                  np.bincount(rows // 256))
            feats = np.where(d[rows].max(0) > 1e-2 * np.abs(b[k]).max())[0]
            print("  bad features", feats[:40], len(feats))
