"""Debug: replicate test_gpu_c3's schedule; check whether the snapshots or the inputs change."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np, torch
from deepinteract_amd import synth
from deepinteract_amd.builder import build_graph_batch
from deepinteract_amd.engine import GeoTEngine, PairTensorOp
from deepinteract_amd.graph import select_graphs
from deepinteract_amd.weights import seeded_state_dict
M, N_RES, K, N_MB = 8, 1000, 20, 3
sd = seeded_state_dict(0, with_head=False)
eng = GeoTEngine(sd, "bf16")
n_cx = M * N_MB
chains = [c for j in range(n_cx) for c in synth.synthetic_complex(700 + j, N_RES, N_RES)]
pool = build_graph_batch(chains, k=K, nbr_seeds=list(range(1, 2 * n_cx + 1)))
mbs = [select_graphs(pool, range(2 * M * m, 2 * M * (m + 1))) for m in range(N_MB)]
torch.cuda.synchronize()
snap = [{k: getattr(gb, k).clone() for k in ("src", "dst", "nbr", "node_f", "edge_f", "in_ptr", "node_pos")} for gb in mbs]
torch.cuda.synchronize()
gb0 = mbs[0]
h1r = [gb0.node_off[2 * j] for j in range(M)]
h2r = [gb0.node_off[2 * j + 1] for j in range(M)]
l1 = l2 = [N_RES] * M
mode = sys.argv[1] if len(sys.argv) > 1 else "vector"
pair = PairTensorOp(kernel="vector" if mode == "vector" else "rows")
s_geot = torch.cuda.current_stream(); s_pair = torch.cuda.Stream()
done, keep = [None, None], []
for m, gb in enumerate(mbs):
    slot = m & 1
    with torch.cuda.stream(s_geot):
        if done[slot] is not None:
            s_geot.wait_event(done[slot])
        h, e = eng.forward(gb, clone=False, slot=slot)
        hT = eng.last_hT
        ready = torch.cuda.Event(); ready.record(s_geot)
    with torch.cuda.stream(s_pair):
        s_pair.wait_event(ready)
        if mode != "nopair":
            out, views = pair(h, h1r, h2r, l1, l2, hT=hT)
        hc, ec = h.clone(), e.clone()
        ev = torch.cuda.Event(); ev.record(s_pair); done[slot] = ev
    keep.append((hc, ec))
torch.cuda.synchronize()
for m, gb in enumerate(mbs):
    for k_, v in snap[m].items():
        if not torch.equal(getattr(gb, k_), v):
            d = (getattr(gb, k_) != v).nonzero()
            print(f"INPUT CHANGED mb{m} {k_}: {d.shape[0]} entries, first {d[:4].tolist()}")
# serial recompute
eng2 = GeoTEngine(sd, "bf16")
for m, gb in enumerate(mbs):
    h, e = eng2.forward(gb)
    torch.cuda.synchronize()
    hc, ec = keep[m]
    dh = (h.float() - hc.float()).abs().max().item(); de = (e.float() - ec.float()).abs()
    rows = (de.max(1).values > 0).nonzero().flatten()
    print(f"mb{m} [{mode}]: node maxdiff {dh:.3e}, edge maxdiff {de.max().item():.3e}, differing edge rows {rows.numel()}",
          rows[:10].tolist(), rows[-5:].tolist() if rows.numel() else "")
