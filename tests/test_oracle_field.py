"""Oracle f128 arithmetic (winter-math 0.13.1 fields::f128) against Python big ints."""
import random

P = 2**128 - 45 * 2**40 + 1
G40 = 23953097886125630542083529559205016746  # TWO_ADIC_ROOT_OF_UNITY (winter-math f128)


def test_constants(oracle):
    assert oracle.P == P
    assert pow(3, (P - 1) // 2**40, P) == G40
    assert oracle.root_of_unity(40) == G40
    for k in (1, 5, 16, 20):
        w = oracle.root_of_unity(k)
        assert pow(w, 2**k, P) == 1 and pow(w, 2**(k - 1), P) != 1


def test_random_ops(oracle):
    rng = random.Random(7)
    edge = [0, 1, 2, P - 1, P - 2, 2**64, 2**64 - 1, 2**127, P - 2**64, 45 * 2**40 - 1]
    vals = edge + [rng.randrange(P) for _ in range(300)]
    for i in range(len(vals)):
        a, b = vals[i], vals[(i * 7 + 3) % len(vals)]
        assert oracle.fe_add(a, b) == (a + b) % P
        assert oracle.fe_sub(a, b) == (a - b) % P
        assert oracle.fe_mul(a, b) == (a * b) % P
        if a:
            assert oracle.fe_mul(oracle.fe_inv(a), a) == 1
