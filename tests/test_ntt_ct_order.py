"""The index algebra of ntt_ct_lazy_kernel (kernels.hip): a natural -> bit-reversed transform as
Cooley-Tukey butterflies in decreasing-stride order, where the butterfly of block b at global half
size H (m = N / 2H blocks) takes w_(2m)^brv(b), equals the Gentleman-Sande DIF transform the
canonical kernel computes -- for every split into passes of r stages at stride S, with the kernel's
own group / quad coordinates.  Modelled over a small NTT prime (the algebra does not depend on the
field); the device kernel itself is pinned by the GPU NTT / LDE / proof tests."""
import random

import pytest

P, GEN = 998244353, 3


def _brv(x, bits):
    r = 0
    for i in range(bits):
        r = (r << 1) | ((x >> i) & 1)
    return r


def _root(n):
    return pow(GEN, (P - 1) // n, P)


def _dif(x):
    n, a, h = len(x), list(x), len(x) // 2
    while h >= 1:
        w = _root(2 * h)
        for s in range(0, n, 2 * h):
            for j in range(h):
                u, v = a[s + j], a[s + j + h]
                a[s + j], a[s + j + h] = (u + v) % P, (u - v) * pow(w, j, P) % P
        h //= 2
    return a


def _ct_passes(x, rs):
    """ntt_passes(dif=True) with ntt_ct_lazy_kernel: passes in rs (ascending stride) walked from the
    largest stride; inside a pass the quads (lh, lh-1) and a last single stage, as the kernel."""
    n = len(x)
    log_n = n.bit_length() - 1
    a = list(x)
    cur = log_n - 1
    for r in reversed(rs):
        log_s = cur - r + 1
        S, R = 1 << log_s, 1 << r
        for q in range(n >> r):
            L, hb = q & (S - 1), q >> log_s
            idx = [hb * S * R + t * S + L for t in range(R)]
            loc = [a[i] for i in idx]

            def tw(lh, t0):
                logm = log_n - 1 - lh - log_s
                b = hb * (R >> (lh + 1)) + (t0 >> (lh + 1))
                return pow(_root(2 << logm), _brv(b, logm), P)

            def bfly(i, j, w):
                v = loc[j] * w % P
                loc[i], loc[j] = (loc[i] + v) % P, (loc[i] - v) % P

            lh = r - 1
            while lh >= 1:
                hl = 1 << (lh - 1)
                for w in range(R // 4):
                    k = w & (hl - 1)
                    t0 = ((w >> (lh - 1)) << (lh + 1)) + k
                    w1, w2, w3 = tw(lh, t0), tw(lh - 1, t0), tw(lh - 1, t0 + 2 * hl)
                    bfly(t0, t0 + 2 * hl, w1)
                    bfly(t0 + hl, t0 + 3 * hl, w1)
                    bfly(t0, t0 + hl, w2)
                    bfly(t0 + 2 * hl, t0 + 3 * hl, w3)
                lh -= 2
            if lh == 0:
                for u in range(R // 2):
                    t0 = u << 1
                    bfly(t0, t0 + 1, tw(0, t0))
            for i, t in zip(idx, range(R)):
                a[i] = loc[t]
        cur -= r
    return a


@pytest.mark.parametrize("log_n,rs", [(4, [4]), (5, [2, 3]), (6, [3, 3]), (8, [8]), (9, [8, 1]), (10, [2, 8]),
                                      (11, [8, 3]), (12, [1, 3, 8])])
def test_ct_decreasing_stride_equals_dif(log_n, rs):
    rng = random.Random(log_n * 131 + len(rs))
    x = [rng.randrange(P) for _ in range(1 << log_n)]
    assert _ct_passes(x, rs) == _dif(x)
