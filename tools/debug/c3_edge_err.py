"""Debug: locate the C3 bf16 edge-output outliers of test_gpu_c3 (pool chain 0)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import numpy as np, torch
from deepinteract_amd import synth
from deepinteract_amd.builder import build_graph_batch
from deepinteract_amd.engine import GeoTEngine
from deepinteract_amd.graph import select_graphs
from deepinteract_amd.weights import seeded_state_dict
from oracle import geot_oracle as O

def og(gb, g):
    n0, n1 = gb.node_off[g], gb.node_off[g + 1]; e0, e1 = gb.edge_off[g], gb.edge_off[g + 1]
    nbr = gb.nbr[e0:e1].long().cpu() - e0
    return {"num_nodes": n1 - n0, "src": gb.src[e0:e1].long().cpu() - n0, "dst": gb.dst[e0:e1].long().cpu() - n0,
            "src_nbr": nbr[:, :2], "dst_nbr": nbr[:, 2:], "node_f": gb.node_f[n0:n1].cpu(), "edge_f": gb.edge_f[e0:e1].cpu()}

sd = seeded_state_dict(0, with_head=False)
chains = [c for j in range(8) for c in synth.synthetic_complex(700 + j, 1000, 1000)]
pool = build_graph_batch(chains, k=20, nbr_seeds=list(range(1, 17)))
nbr = pool.nbr.cpu().numpy(); src = pool.src.cpu().numpy(); dst = pool.dst.cpu().numpy()
print("nbr range checks:", (nbr[:, :2] // 20 == src[:, None]).all(), (nbr[:, 2:] // 20 == dst[:, None]).all())
g = og(pool, 0)
with torch.no_grad():
    n_ref, e_ref, inter = O.geot_forward(sd, g, return_intermediates=True)
e_ref = e_ref.numpy(); n_ref = n_ref.numpy()
for name, dt, sel in (("bf16 batch16", "bf16", None), ("f32 batch16", "f32", None), ("bf16 alone", "bf16", [0])):
    eng = GeoTEngine(sd, dt)
    gb = pool if sel is None else select_graphs(pool, sel)
    h, e = eng.forward(gb)
    torch.cuda.synchronize()
    e0 = e[:20000].float().cpu().numpy(); h0 = h[:1000].float().cpu().numpy()
    err = np.abs(e0 - e_ref).max(1) / np.abs(e_ref).max()
    bad = np.argsort(-err)[:8]
    print(name, "node rel", np.abs(h0 - n_ref).max() / np.abs(n_ref).max(), "edge rel", err.max())
    print("  worst edges", bad.tolist(), err[bad].round(4).tolist())
    print("  |ref| of worst", np.abs(e_ref[bad]).max(1).round(2).tolist(), "max|ref|", np.abs(e_ref).max().round(2))
    print("  src/dst of worst", src[bad].tolist(), dst[bad].tolist())
