"""The persistent engine's host-checkable invariants (CPU only).

Ticket groups: ticket t goes to group t % 8, which the
waves of workgroups w % 8 == group take; the group comes from the workgroup
index, not the hardware XCC id (which on a partitioned or smaller device may
miss values and leave tickets unclaimed).  The arithmetic the kernel runs is
the host-callable code in crc32c_internal.hpp, reached through the
diagnostics library's nova_diag_engine_groups (no GPU needed).
"""
import ctypes

import numpy as np
import pytest

from novalsm_amd import crc32c as C


@pytest.fixture(scope="module")
def diag():
    C.load(build_if_missing=True)
    return C.load_diag()


def _groups(D, wgs, cs, ce):
    out = (ctypes.c_uint64 * 17)()
    assert D.nova_diag_engine_groups(wgs, cs, ce, out) == 0
    v = [int(x) for x in out]
    return v[:8], v[8:16], v[16]


@pytest.mark.parametrize("wgs", [8, 16, 24, 32, 64, 128, 248, 256, 512])
def test_every_group_has_workgroups(diag, wgs):
    """Any engine grid (at least 8 workgroups, a multiple of 8: NOVA_SST_ENGINE_CUS
    rounds down to one) gives every group the same number of workgroups."""
    per, _, _ = _groups(diag, wgs, 0, 0)
    assert per == [wgs // 8] * 8


def test_request_tickets_split_over_groups(diag):
    """A request's tickets [cstart, cend) split over the groups exactly (the
    per-group completion lines sum to the request), every group with tickets
    counts toward completion, and no group without tickets does."""
    rng = np.random.default_rng(3)
    cases = [(0, 0), (0, 1), (0, 7), (0, 8), (0, 9), (5, 6), (7, 16), (1, 1025)]
    cases += [(int(a), int(a + b)) for a, b in zip(rng.integers(0, 1 << 40, 300), rng.integers(0, 5000, 300))]
    for cs, ce in cases:
        _, share, used = _groups(diag, 256, cs, ce)
        assert sum(share) == ce - cs, (cs, ce, share)
        want = [sum(1 for t in range(cs, min(ce, cs + 64)) if t % 8 == g) for g in range(8)] \
            if ce - cs <= 64 else None
        if want is not None:
            assert share == want, (cs, ce)
        assert used == sum(1 for x in share if x), (cs, ce, share)
        assert max(share) - min(share) <= 1

