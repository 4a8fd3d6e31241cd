"""Oracle prover self-consistency: boundary-term forms agree, proofs are deterministic."""
import hashlib

import pytest


@pytest.mark.parametrize("log_n", [5, 7])
def test_boundary_forms_agree(oracle, log_n):
    t, pi, w = oracle.synth_segment(0x5EED0002, log_n)
    n = 1 << log_n
    opts = oracle.default_options(w, n, queries=16, grind=2)
    a = oracle.prove(t, w, n, pi, opts, boundary_mode=0)
    b = oracle.prove(t, w, n, pi, opts, boundary_mode=1)
    assert a == b


def test_deterministic_and_seed_sensitive(oracle):
    t, pi, w = oracle.synth_segment(0x5EED0003, 5)
    opts = oracle.default_options(w, 32, queries=8, grind=4)
    a = oracle.prove(t, w, 32, pi, opts)
    assert a == oracle.prove(t, w, 32, pi, opts)
    t2, pi2, _ = oracle.synth_segment(0x5EED0004, 5)
    assert a != oracle.prove(t2, w, 32, pi2, opts)
