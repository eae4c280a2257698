"""Run one C3 micro-batch through the stamped edge kernels (tools/diag/build_stamps.py) and print
per-stage cycle statistics: 'wait' = cycles inside EdgeStages::next() (weight stage not ready /
barrier), 'work' = cycles from leaving next() to reaching the following one. usage:
python tools/diag/run_stamps.py <variant lib> [serial]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from deepinteract_amd import _lib, synth  # noqa: E402

lib = _lib.load_variant(sys.argv[1])
from deepinteract_amd.builder import build_graph_batch  # noqa: E402
from deepinteract_amd.engine import GeoTEngine  # noqa: E402
from deepinteract_amd.weights import seeded_state_dict  # noqa: E402

buf = torch.zeros(64 * 8 * 192, dtype=torch.int64, device="cuda")
chains = [c for j in range(8) for c in synth.synthetic_complex(900 + j, 1000, 1000)]
gb = build_graph_batch(chains, nbr_seeds=list(range(16)))
eng = GeoTEngine(seeded_state_dict(0, with_head=False), "bf16")
for _ in range(3):
    eng.forward(gb, clone=False)
torch.cuda.synchronize()
fn = getattr(lib, "di_diag_stamps")
fn.argtypes = [ctypes.c_void_p]
for label in ("intermediate", "final"):
    buf.zero_()
    assert fn(ctypes.c_void_p(buf.data_ptr())) == 0
    # run only the edge layer of interest: full forward, stamps overwritten by the later launch;
    # so run the forward and read the FINAL layer's stamps, or stop after layer 0 for intermediate
    eng.forward(gb, clone=False)
    torch.cuda.synchronize()
    assert fn(ctypes.c_void_p(0)) == 0
    t = buf.view(64, 8, 64, 3).cpu().numpy().astype(np.int64)
    ok = (t[..., 0] > 0) & (t[..., 1] > 0) & (t[..., 2] > 0)
    nst = int(ok[0, 0].sum())
    wait = t[..., 1] - t[..., 0]
    iss = t[..., 2] - t[..., 1]
    work = np.zeros_like(wait)
    work[..., :-1] = t[:, :, 1:, 0] - t[:, :, :-1, 2]
    okw = ok.copy()
    okw[..., :-1] &= ok[..., 1:]
    okw[..., -1] = False
    print(f"== stamps of the LAST edge launch, {nst} stages recorded for wave 0 of block 0")
    print("stage  wait(med,p90)   issue(med,p90)   work(med,p90)")
    for s_ in range(min(nst, 64)):
        m = ok[:, :, s_]
        if not m.any():
            continue
        w, q = wait[:, :, s_][m], iss[:, :, s_][m]
        k = work[:, :, s_][okw[:, :, s_]]
        print(f"{s_:5d}  {int(np.median(w)):6d} {int(np.percentile(w, 90)):6d}   {int(np.median(q)):6d} "
              f"{int(np.percentile(q, 90)):6d}   {int(np.median(k)) if k.size else 0:6d} "
              f"{int(np.percentile(k, 90)) if k.size else 0:6d}")
    tw, tq, tk = wait[ok].sum(), iss[ok].sum(), work[okw].sum()
    tot = tw + tq + tk
    print(f"share of stamped cycles: wait {tw / tot:.1%}, DMA issue {tq / tot:.1%}, work {tk / tot:.1%}")
    break
