"""Host-side configuration checks of the overlapped schedule (no GPU: they fire before any stream or
buffer is created)."""
import types

import pytest

from deepinteract_amd.pipeline import OverlappedSchedule


def _eng(dtype="bf16", fuse=True, resident=True):
    return types.SimpleNamespace(dtype=dtype, fuse_embed_init=fuse, resident_init=resident)


def test_resident_init_edge_is_refused_beside_the_pair_stream():
    # the LDS-resident InitEdge block (3 x 168 VGPRs per SIMD) cannot share a SIMD with a pair-stream
    # wave; with a store wave on every CU the pair stream would give up on every wave
    with pytest.raises(ValueError, match="resident InitEdge"):
        OverlappedSchedule(_eng(fuse=False, resident=True), [], [], [], [], [], [])


def test_ring_must_cover_two_help_periods():
    with pytest.raises(ValueError, match="ring >= 2"):
        OverlappedSchedule(_eng(), [], [], [], [], [], [], ring=6, help_every=4)
