"""Dense CPU emulation of the GeoT kernels' dataflow, driven by the PACKED weight blobs.

Test infrastructure: it reads the exact blobs the HIP kernels read (same offsets as
csrc/layout.h), unpacks them, and replays each kernel's per-row program in float64. Comparing it
with the oracle checks the host packing, BatchNorm folding, pre-multiplied geometric
embeddings and layout offsets on CPU, before any GPU run.
"""
import numpy as np
import torch

from deepinteract_amd import packing


def _unpack(mat, off, nout, kin, dtype, layout=16):
    """W [nout, kin] from the packed blocks at block offset `off` (16-row or 32-row fragment order)."""
    flat = mat.to(torch.float64).numpy()
    W = np.zeros((nout, kin))
    if layout == 32:
        r, c = packing._pack_index32()
        rows, cols = 32, 16
    else:
        r, c = packing._pack_index(dtype)
        rows, cols = 16, 32
    nbo, ns = nout // rows, kin // cols
    for bo in range(nbo):
        for s in range(ns):
            k = off + bo * ns + s
            W[rows * bo + r, cols * s + c] = flat[k * 512:(k + 1) * 512]
    return W


def silu(x):
    return x / (1.0 + np.exp(-x))


def silu2(x):
    """log2-unit SiLU of the bf16 kernels (csrc/common.h): x * sigmoid(x * ln 2)."""
    return x / (1.0 + np.exp2(-x))


class Emu:
    def __init__(self, packed: packing.PackedGeoT):
        self.p, self.dt = packed, packed.dtype
        self.s2 = silu2 if packed.dtype == "bf16" else silu
        self.u = np.log(2.0) if packed.dtype == "bf16" else 1.0  # silu = silu2 * u

    def M(self, blob, off, nout, kin):
        if any(blob is e for e in self.p.edge):
            layout = self.p.edge_layout
        elif blob is self.p.init:
            layout = self.p.init_layout
        else:
            layout = 16
        return _unpack(blob[0], off, nout, kin, self.dt, layout)

    def geot(self, g):
        """g: dict with num_nodes, src, dst, node_f, edge_f, src_nbr, dst_nbr (torch)."""
        p = self.p
        src, dst = g["src"].numpy(), g["dst"].numpy()
        N, E = g["num_nodes"], src.size
        nbr = np.concatenate([g["src_nbr"].numpy(), g["dst_nbr"].numpy()], 1)
        G = np.zeros((E, 32))
        G[:, :28] = g["edge_f"].numpy()
        xn = np.zeros((N, 128))
        xn[:, :113] = g["node_f"].numpy()
        # embed
        em, ev = p.embed[0], p.embed[1].numpy()
        h = xn @ self.M(p.embed, 0, 128, 128).T
        qkv = np.concatenate([h @ self.M(p.embed, 32 + 32 * i, 128, 128).T + ev[128 * i:128 * i + 128]
                              for i in range(3)], 1)
        # init edge
        ib = p.init
        pos = np.arange(N)  # per-chain graph
        acc = p.pos_src.numpy()[pos[src]] + p.pos_dst.numpy()[pos[dst]]
        s2 = self.s2
        acc = acc + G @ self.M(ib, 0, 128, 32).T  # t = 0: collapsed edge-message map
        for t in range(1, 5):
            y = s2(G @ self.M(ib, 40 * t, 128, 32).T)
            acc = acc + y @ self.M(ib, 40 * t + 8, 128, 128).T
        c = s2(acc)
        gs = sum((G @ self.M(ib, 200 + 8 * t, 128, 32).T) if t == 0 else s2(G @ self.M(ib, 200 + 8 * t, 128, 32).T)
                 for t in range(5))
        c = c * gs
        z = c @ self.M(ib, 240, 32, 128).T
        F = z @ self.M(ib, 248, 128, 32).T
        Fn = silu(F @ self.M(ib, 256, 128, 128).T + ib[1].numpy()[:128])  # stored post-activation
        L = p.num_layers
        F_last = F
        for li in range(L):
            final = li == L - 1
            eb = p.edge[li]
            V = eb[1].numpy()
            mg = self.M(eb, 0, 320, 32)
            fgm = self.M(eb, 532, 128, 32)
            gate = (G @ mg[128:192].T) * (G @ mg[192:256].T) * (G @ mg[256:320].T)
            dg = G @ mg[0:128].T
            Wd = self.M(eb, 20, 64, 128)
            s = 0
            for j in range(4):
                x = Fn[nbr[:, j]] * dg
                s = s + s2(x @ Wd.T) * gate
            u = self.u
            x = u * s2(s @ self.M(eb, 36, 128, 64).T) + V[0:128] + F @ self.M(eb, 52, 128, 128).T
            for rb in range(4):
                if rb == 2:
                    x = F + u * s2(x @ self.M(eb, 468, 128, 128).T + V[1664:1792])
                y = x
                for l in range(3):
                    i = 3 * rb + l
                    y = s2(y @ self.M(eb, 84 + 32 * i, 128, 128).T + V[128 + 128 * i:256 + 128 * i])
                x = x + u * y
            x = x * (G @ fgm.T)
            conf = F + u * s2(x @ self.M(eb, 500, 128, 128).T + V[1792:1920])
            P = conf @ self.M(eb, 540, 128, 128).T + V[1920:2048]
            sc = np.clip(qkv[src, 128:256] * qkv[dst, 0:128] / np.sqrt(32), -5, 5) * P
            alpha = np.exp(np.clip(sc.reshape(E, 4, 32).sum(-1), -5, 5))
            if not final:
                e1 = F + sc @ self.M(eb, 572, 128, 128).T + V[2048:2176]
                o = 0
                for half in range(2):
                    t_ = s2(e1 @ self.M(eb, 604 + 32 * half, 128, 128).T + V[2176 + 128 * half:2304 + 128 * half])
                    o = o + t_ @ self.M(eb, 668 + 32 * half, 128, 128).T
                F_next = e1 + o
                Fn = silu(F_next @ self.M(eb, 732, 128, 128).T + V[2432:2560])
            # node layer
            nb = p.node[li]
            NV = nb[1].numpy()
            wv = np.zeros((N, 4, 32))
            z = np.zeros((N, 4))
            np.add.at(wv, dst, alpha[:, :, None] * qkv[src, 256:384].reshape(E, 4, 32))
            np.add.at(z, dst, alpha)
            hatt = (wv / (z[:, :, None] + 1e-6)).reshape(N, 128)
            n = h + hatt @ self.M(nb, 0, 128, 128).T + NV[0:128]
            o = 0
            for half in range(2):
                t_ = s2(n @ self.M(nb, 32 + 32 * half, 128, 128).T + NV[128 + 128 * half:256 + 128 * half])
                o = o + t_ @ self.M(nb, 96 + 32 * half, 128, 128).T
            h = n + o
            if not final:
                qkv = np.concatenate([h @ self.M(nb, 160 + 32 * i, 128, 128).T + NV[384 + 128 * i:512 + 128 * i]
                                      for i in range(3)], 1)
                F = F_next
                F_last = F_next
        return h, F_last
