"""The torch-seeded neighbour-edge ids (csrc/graph_builder.hip k_nbr_ids_torch): a Python mirror
of the kernel's arithmetic — mt19937 seeding, the twist in the kernel's three data-parallel
phases, tempering, and the closed form of the first two Fisher-Yates draws — against
torch.randperm (the reference's call, deepinteract_utils.py:539-546) and against the neighbour ids
the reference's own convert_df_to_dgl_graph produced for the golden fixtures."""
import numpy as np
import pytest
import torch

from gpu_common import load_case

N, M = 624, 397


def mt_init(seed):
    st = np.zeros(N, dtype=np.uint64)
    s = seed & 0xffffffff
    st[0] = s
    for i in range(1, N):
        s = (1812433253 * (s ^ (s >> 30)) + i) & 0xffffffff
        st[i] = s
    return st.astype(np.uint32)


def _next(cur, nxt, far):
    y = (cur & np.uint32(0x80000000)) | (nxt & np.uint32(0x7fffffff))
    return far ^ (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), np.uint32(0x9908b0df), np.uint32(0))


def mt_twist_phased(st):
    """The kernel's twist: [0,227) from old words; [227,454) reads phase-1 words; [454,624)
    reads phase-2 words and the new word 0."""
    st = st.copy()
    a = np.arange(0, N - M)
    st[a] = _next(st[a], st[a + 1], st[a + M])
    b = np.arange(N - M, 2 * (N - M))
    st[b] = _next(st[b], st[b + 1], st[b - (N - M)])
    c = np.arange(2 * (N - M), N)
    st[c] = _next(st[c], st[(c + 1) % N], st[c - (N - M)])
    return st


def temper(y):
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9d2c5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xefc60000))
    return y ^ (y >> np.uint32(18))


def stream(seed, count):
    st, out = mt_init(seed), []
    while len(out) * N < count:
        st = mt_twist_phased(st)
        out.append(temper(st))
    return np.concatenate(out)[:count]


def kept_draws(seed, E, k):
    """(src_side [E,2], dst_side [E,2]) permutation prefixes, as the kernel computes them."""
    u = stream(seed, 2 * E * (k - 1)).astype(np.int64).reshape(2 * E, k - 1)
    z0 = u[:, 0] % k
    z1 = u[:, 1] % (k - 1)
    p1 = np.where(1 + z1 == z0, 0, 1 + z1)
    p = np.stack([z0, p1], 1)
    return p[:E], p[E:]


@pytest.mark.parametrize("seed", [0, 7, 101, 2 ** 31 + 5])
@pytest.mark.parametrize("k", [20, 30])
def test_phased_mt19937_prefixes_match_torch_randperm(seed, k):
    E = 700  # crosses many 624-word blocks, incl. draws split across a block boundary
    ps, pd = kept_draws(seed, E, k)
    g = torch.Generator().manual_seed(seed)
    ref = np.stack([torch.randperm(k, generator=g)[:2].numpy() for _ in range(2 * E)])
    assert np.array_equal(ps, ref[:E]) and np.array_equal(pd, ref[E:])


@pytest.mark.parametrize("case", ["tiny", "c1"])
def test_prefixes_reproduce_reference_fixture_ids(case):
    """The fixture's ids came from the reference's own builder after torch.manual_seed(seed)."""
    z = load_case(case)
    k = 20
    for tag in ("g1", "g2"):
        src, dst = z[f"{tag}_src"].astype(np.int64), z[f"{tag}_dst"].astype(np.int64)
        ps, pd = kept_draws(int(z[f"{tag}_nbr_seed"]), src.size, k)
        assert np.array_equal(src[:, None] * k + ps, z[f"{tag}_src_nbr"])
        assert np.array_equal(dst[:, None] * k + pd, z[f"{tag}_dst_nbr"])
