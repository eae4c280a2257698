"""Chain inputs for the graph builder: synthetic (seeded) chains and a minimal PDB reader.

A *chain* is a dict of host numpy arrays:
  backbone   [N,4,3] f32  N, CA, C, O coordinates (deepinteract_utils.py:460-472 layout)
  amide_norm [N,3]   f32  DIPS-Plus amide-plane normal cross(CA-CB, CB-N), zero when CB is
                          missing (dips_plus_utils.py:356-374, zero imputation :908-909)
  dips       [N,106] f32  DIPS-Plus residue features in node-feature column order
                          (resname one-hot 20, ss one-hot 8, rsa, rd, psaia 6, hsaac 42, cn,
                          sequence_feats 27; deepinteract_constants.py:64-96)

Synthetic protocol: complex c, chain s -> numpy Generator seeded 10_000*c + s;
Cα self-avoiding random walk (3.8 Å steps, ≥3.0 Å non-bonded), N/C/O/CB at fixed local
offsets + N(0, 0.05 Å) noise; homodimers are a random rigid transform of chain 1.
"""
from __future__ import annotations

import numpy as np

RESNAMES = ["TRP", "PHE", "LYS", "PRO", "ASP", "ALA", "ARG", "CYS", "VAL", "THR",
            "GLY", "SER", "HIS", "LEU", "GLU", "TYR", "ILE", "ASN", "MET", "GLN"]
SS_VALUES = ['H', 'B', 'E', 'G', 'I', 'T', 'S', '-']
GLY = RESNAMES.index("GLY")

# local-frame offsets (Å) of N, C, O, CB relative to CA; frame axes: (t, n, b)
_LOCAL = {
    "N": np.array([-0.53, 1.36, 0.0]),
    "C": np.array([0.52, -0.20, 1.42]),
    "O": np.array([1.20, -1.20, 1.50]),
    "CB": np.array([-0.52, -0.78, -1.20]),
}


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def random_walk_ca(n: int, rng: np.random.Generator, step=3.8, min_dist=3.0, max_tries=200):
    ca = np.zeros((n, 3), dtype=np.float64)
    for i in range(1, n):
        for _ in range(max_tries):
            d = rng.normal(size=3)
            d /= np.linalg.norm(d)
            cand = ca[i - 1] + step * d
            if i < 2 or np.min(np.sum((ca[:i - 1] - cand) ** 2, axis=1)) >= min_dist ** 2:
                break
        ca[i] = cand
    return ca


def _frames(ca):
    n = ca.shape[0]
    prev = np.concatenate([ca[:1] - (ca[1:2] - ca[:1]), ca[:-1]])
    nxt = np.concatenate([ca[1:], ca[-1:] + (ca[-1:] - ca[-2:-1])])
    t = _unit(nxt - prev)
    side = _unit((ca - prev) - (nxt - ca) + 1e-9)
    nvec = _unit(side - np.sum(side * t, -1, keepdims=True) * t)
    b = np.cross(t, nvec)
    return np.stack([t, nvec, b], axis=1)  # [n,3(axis),3]


def synthetic_chain(n: int, seed: int, ca: np.ndarray | None = None):
    rng = np.random.default_rng(seed)
    if ca is None:
        ca = random_walk_ca(n, rng)
    fr = _frames(ca)
    atoms = {}
    for name, off in _LOCAL.items():
        pos = ca + np.einsum("k,nkd->nd", off, fr)
        atoms[name] = pos + rng.normal(scale=0.05, size=pos.shape)
    ca_noisy = ca + rng.normal(scale=0.05, size=ca.shape)
    backbone = np.stack([atoms["N"], ca_noisy, atoms["C"], atoms["O"]], axis=1)
    resid = rng.integers(0, 20, size=n)
    ss = rng.integers(0, 8, size=n)
    dips = np.zeros((n, 106), dtype=np.float64)
    dips[np.arange(n), resid] = 1.0
    dips[np.arange(n), 20 + ss] = 1.0
    dips[:, 28:] = rng.random((n, 78))
    amide = np.cross(ca_noisy - atoms["CB"], atoms["CB"] - atoms["N"])
    amide[resid == GLY] = 0.0
    return {
        "backbone": backbone.astype(np.float32),
        "amide_norm": amide.astype(np.float32),
        "dips": dips.astype(np.float32),
    }


def random_rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    a, b, c, d = q
    return np.array([[a * a + b * b - c * c - d * d, 2 * (b * c - a * d), 2 * (b * d + a * c)],
                     [2 * (b * c + a * d), a * a - b * b + c * c - d * d, 2 * (c * d - a * b)],
                     [2 * (b * d - a * c), 2 * (c * d + a * b), a * a - b * b - c * c + d * d]])


def rigid_copy(chain, seed: int, shift=30.0):
    rng = np.random.default_rng(seed)
    R = random_rotation(rng)
    t = rng.normal(size=3) * shift
    bb = chain["backbone"].astype(np.float64) @ R.T + t
    am = chain["amide_norm"].astype(np.float64) @ R.T
    return {"backbone": bb.astype(np.float32), "amide_norm": am.astype(np.float32),
            "dips": chain["dips"].copy()}


def synthetic_complex(c: int, n1: int, n2: int, homodimer: bool = False):
    """Complex c: chain s seeded 10_000*c + s."""
    ch1 = synthetic_chain(n1, 10_000 * c + 1)
    if homodimer:
        assert n1 == n2
        ch2 = rigid_copy(ch1, 10_000 * c + 2)
    else:
        ch2 = synthetic_chain(n2, 10_000 * c + 2)
    return ch1, ch2


def read_pdb_chain(path: str, seed: int = 0):
    """Backbone + amide normals from a PDB file (ATOM records, fixed columns). DIPS-Plus
    columns are not derivable offline (PSAIA / HH-suite), so they are seeded synthetic."""
    residues = {}
    order = []
    with open(path) as fh:
        for line in fh:
            if not line.startswith("ATOM"):
                continue
            name = line[12:16].strip()
            key = (line[21], line[22:27])
            if key not in residues:
                residues[key] = {"resname": line[17:20]}
                order.append(key)
            residues[key][name] = np.array([float(line[30:38]), float(line[38:46]), float(line[46:54])])
    keep = [k for k in order if all(a in residues[k] for a in ("N", "CA", "C", "O"))]
    bb = np.stack([np.stack([residues[k][a] for a in ("N", "CA", "C", "O")]) for k in keep])
    amide = np.zeros((len(keep), 3))
    for i, k in enumerate(keep):
        r = residues[k]
        if "CB" in r:
            amide[i] = np.cross(r["CA"] - r["CB"], r["CB"] - r["N"])
    rng = np.random.default_rng(seed)
    n = len(keep)
    dips = np.zeros((n, 106))
    for i, k in enumerate(keep):
        rn = residues[k]["resname"]
        dips[i, RESNAMES.index(rn) if rn in RESNAMES else 19] = 1.0
    dips[np.arange(n), 20 + rng.integers(0, 8, size=n)] = 1.0
    dips[:, 28:] = rng.random((n, 78))
    return {"backbone": bb.astype(np.float32), "amide_norm": amide.astype(np.float32),
            "dips": dips.astype(np.float32)}
