"""Oracle Poseidon suite + PoseidonHasher vs the pure-Python restatement (pyref) and fixtures."""
import json
import os
import random

import pyref

GOLD = os.path.join(os.path.dirname(__file__), "golden", "poseidon_vectors.json")


def test_suite_matches_pyref(oracle):
    for sid in (bytes(32), bytes([1] * 32), bytes(range(32))):
        assert oracle.suite(sid) == pyref.suite(sid)


def test_permutation(oracle):
    rng = random.Random(3)
    st = [rng.randrange(pyref.P) for _ in range(12)]
    assert oracle.permute(st) == pyref.permute(st)


def test_hasher_functions(oracle):
    rng = random.Random(11)
    for n in (0, 1, 2, 3, 19, 20, 21, 51, 102):
        e = [rng.randrange(pyref.P) for _ in range(n)]
        assert oracle.hash_elements(e) == pyref.hash_elements(e)
    a, b = rng.randrange(pyref.P), rng.randrange(pyref.P)
    assert oracle.merge(a, b) == pyref.merge(a, b)
    for n in (0, 1, 4, 9, 10, 11):
        ds = [rng.randrange(pyref.P) for _ in range(n)]
        assert oracle.merge_many(ds) == pyref.merge_many(ds)
    assert oracle.merge_with_int(a, 0xDEADBEEF12345678) == pyref.merge_with_int(a, 0xDEADBEEF12345678)
    for n in (0, 5, 32, 33, 100):
        msg = bytes(rng.randrange(256) for _ in range(n))
        assert oracle.hash_bytes(msg) == pyref.hash_bytes(msg)


def test_program_field_commitment(oracle):
    pid = bytes(range(1, 33))
    dom, mds, rc = pyref.suite(pid)
    st = [0] * 12
    st[0] = int.from_bytes(pid[:16], "little") % pyref.P
    st[1] = int.from_bytes(pid[16:], "little") % pyref.P
    st[10], st[11] = dom
    st = pyref.permute(st, (dom, mds, rc))
    assert oracle.program_field_commitment(pid) == (st[0], st[1])


def test_golden_fixture(oracle):
    """Committed vectors (tests/golden/make_golden.py): self-consistency pins of the
    restatement; parity against real Winterfell output is unpinned (no Rust toolchain)."""
    g = json.load(open(GOLD))
    assert oracle.hash_elements(g["hash_elements"]["input"]) == g["hash_elements"]["output"]
    assert oracle.merge(*g["merge"]["input"]) == g["merge"]["output"]
    assert oracle.merge_with_int(*g["merge_with_int"]["input"]) == g["merge_with_int"]["output"]
    assert oracle.suite(bytes(32))[0] == g["hasher_dom"]
