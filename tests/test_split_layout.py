"""Invariants of the split layout of the trace LDE (kernels.h lde_pos / lde_row),
restated in Python: the layout is a permutation of each column, it stays inside the set of
positions one workgroup of the last DIT pass reads (8 consecutive L, all t: the pass stores in
place), even rows fill the first half in whole 8-element lines, and the next row of an even row
sits `blowup` positions further except where its L wraps.  The GPU parity tests prove through
the C++ form of the same functions."""
import pytest


def lde_pos(r, N):
    logS = N.bit_length() - 1 - 8
    S = 1 << logS
    L, t = r & (S - 1), r >> logS
    l = L & 7
    return (L - l) + (l >> 1) + ((t & 1) << 2) + (((t >> 1) + ((l & 1) << 7)) << logS)


def lde_row(q, N):
    logS = N.bit_length() - 1 - 8
    S = 1 << logS
    Lp, tp = q & (S - 1), q >> logS
    m = Lp & 7
    l = ((m & 3) << 1) | (tp >> 7)
    t = ((tp & 127) << 1) | (m >> 2)
    return (Lp - m) + l + (t << logS)


@pytest.mark.parametrize("log_n", [11, 12, 14, 16])
def test_permutation_in_place_and_halves(log_n):
    N = 1 << log_n
    S = N >> 8
    seen = set()
    for r in range(N):
        q = lde_pos(r, N)
        assert 0 <= q < N and q not in seen
        seen.add(q)
        assert lde_row(q, N) == r
        assert ((q & (S - 1)) >> 3) == ((r & (S - 1)) >> 3)  # same workgroup of the last pass
        assert (q < N // 2) == (r % 2 == 0)
    # every aligned line of 8 positions holds rows of one parity
    for q0 in range(0, N, 8):
        assert len({lde_row(q, N) & 1 for q in range(q0, q0 + 8)}) == 1


@pytest.mark.parametrize("blowup", [8, 16, 32])
def test_next_row_offset(blowup):
    N = 1 << 14
    S = N >> 8
    for r in range(0, N, 2):
        if (r & (S - 1)) + blowup < S:
            assert lde_pos(r + blowup, N) == lde_pos(r, N) + blowup
