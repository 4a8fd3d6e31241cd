"""Product-side segment verifier (zkl_verify_segment) on the host: it
accepts the oracle's proofs of every segment layout and option set, rejects corrupted or
mismatched ones, and agrees with the oracle verifier on accept / reject (the GPU proofs it
accepts are checked in tests/test_gpu_parity.py)."""
import ctypes as C
import random

import pytest


def _lib_pi(zkl_hip, opi):
    pi = zkl_hip.AirPublicInputs()
    C.memmove(C.byref(pi), C.byref(opi), C.sizeof(pi))
    return pi


def _lib_opts(zkl_hip, oo):
    return zkl_hip.ProofOptions(*[getattr(oo, f) for f, _ in oo._fields_])


CASES = [  # seed, log_n, flags, q, blowup, grind, partitions
    (0x5EED0B01, 5, 0, 8, 16, 2, 1),
    (0x5EED0B02, 6, 0, 32, 8, 4, 1),
    (0x5EED0B03, 7, 1, 24, 8, 3, 1),     # sponge: PoseidonAir block
    (0x5EED0B04, 8, 2, 16, 16, 2, 2),    # RAM, two partitions
    (0x5EED0B05, 8, 4, 16, 16, 0, 1),    # Merkle
    (0x5EED0B06, 8, 7, 12, 32, 1, 4),    # everything, four partitions
    (0x5EED0B07, 6, 0, 255, 8, 1, 1),    # maximum queries: heavy position collisions
    (0x5EED0B08, 9, 6, 40, 16, 5, 1),
]


@pytest.mark.parametrize("seed,log_n,flags,q,blowup,grind,parts", CASES)
def test_library_verifier_accepts_oracle_proofs(oracle, seed, log_n, flags, q, blowup, grind, parts):
    import zkl_hip
    n = 1 << log_n
    t, opi, w = oracle.synth_segment(seed, log_n, flags)
    oo = oracle.default_options(w, n, queries=q, blowup=blowup, grind=grind)
    oo.num_partitions = parts
    proof = oracle.prove(t, w, n, opi, oo)
    zkl_hip.verify_segment(proof, _lib_pi(zkl_hip, opi), _lib_opts(zkl_hip, oo))


def test_library_verifier_rejects_corruptions_like_the_oracle(oracle):
    """Flip one byte at 200 positions spread over the proof: the library verifier and the
    oracle verifier give the same verdict each time (almost always: reject)."""
    import zkl_hip
    n = 64
    t, opi, w = oracle.synth_segment(0x5EED0B10, 6, 0)
    oo = oracle.default_options(w, n, queries=16, blowup=8, grind=2)
    proof = oracle.prove(t, w, n, opi, oo)
    pi, o = _lib_pi(zkl_hip, opi), _lib_opts(zkl_hip, oo)
    rng = random.Random(3)
    rejected = 0
    for k in range(200):
        b = bytearray(proof)
        i = rng.randrange(len(b)) if k % 4 else (k * 7919) % len(b)
        b[i] ^= 1 << rng.randrange(8)
        want = oracle.verify(bytes(b), opi, oo)[0] == 0
        try:
            zkl_hip.verify_segment(bytes(b), pi, o)
            got = True
        except zkl_hip.ZklError:
            got = False
        assert got == want, f"byte {i}"
        rejected += not got
    assert rejected >= 190
    with pytest.raises(zkl_hip.ZklError, match="malformed|trailing"):
        zkl_hip.verify_segment(proof + b"\0", pi, o)
    with pytest.raises(zkl_hip.ZklError):
        zkl_hip.verify_segment(proof[:-9], pi, o)


@pytest.mark.parametrize("what,msg", [
    ("pc_init", "identity"), ("queries", "options"), ("rule", "constraint Merkle opening"),
])
def test_library_verifier_rejects_mismatched_statement(oracle, what, msg):
    import zkl_hip
    n = 64
    t, opi, w = oracle.synth_segment(0x5EED0B11, 6, 0)
    oo = oracle.default_options(w, n, queries=16, blowup=8, grind=0)
    oo.num_partitions = 2
    proof = oracle.prove(t, w, n, opi, oo)
    pi, o = _lib_pi(zkl_hip, opi), _lib_opts(zkl_hip, oo)
    if what == "pc_init":
        pi.pc_init.lo ^= 1
    elif what == "queries":
        o.num_queries += 1
    if what == "rule":
        with zkl_hip.row_digest_rule(1), pytest.raises(zkl_hip.ZklError, match=msg):
            zkl_hip.verify_segment(proof, pi, o)
    else:
        with pytest.raises(zkl_hip.ZklError, match=msg):
            zkl_hip.verify_segment(proof, pi, o)
