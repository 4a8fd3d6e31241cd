"""Oracle verifier: proofs from the oracle prover verify; any single
corrupted field, wrong public input or wrong option is rejected with the failing check."""
import random

import pytest


def _prove(oracle, seed, log_n, **kw):
    n = 1 << log_n
    t, pi, w = oracle.synth_segment(seed, log_n)
    opts = oracle.default_options(w, n, **kw)
    return oracle.prove(t, w, n, pi, opts), pi, opts


@pytest.mark.parametrize("log_n,q,blowup,grind", [(5, 8, 16, 0), (6, 32, 8, 4), (7, 20, 32, 6), (8, 64, 16, 8)])
def test_oracle_proofs_verify(oracle, log_n, q, blowup, grind):
    proof, pi, opts = _prove(oracle, 0x5EED0001 + log_n, log_n, queries=q, blowup=blowup, grind=grind)
    rc, err = oracle.verify(proof, pi, opts)
    assert rc == 0, err


def test_corrupted_proofs_rejected(oracle):
    proof, pi, opts = _prove(oracle, 0x5EED0042, 6, queries=16, grind=4)
    assert oracle.verify(proof, pi, opts)[0] == 0
    rng = random.Random(3)
    # flip one bit at positions spread over every section of the proof
    positions = sorted({rng.randrange(len(proof)) for _ in range(60)} | {0, 3, 30, len(proof) - 1})
    accepted = []
    for p in positions:
        bad = bytearray(proof)
        bad[p] ^= 1 << rng.randrange(8)
        rc, err = oracle.verify(bytes(bad), pi, opts)
        if rc == 0:
            accepted.append(p)
    assert not accepted, f"corruptions at {accepted} accepted"
    assert oracle.verify(proof[:-1], pi, opts)[0] != 0
    assert oracle.verify(proof + b"\0", pi, opts)[0] != 0


def test_wrong_public_inputs_rejected(oracle):
    proof, pi, opts = _prove(oracle, 0x5EED0043, 6, queries=16, grind=4)
    pi.pc_init.lo ^= 1
    rc, err = oracle.verify(proof, pi, opts)
    assert rc != 0
    assert err
