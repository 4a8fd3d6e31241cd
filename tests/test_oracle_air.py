"""ZkLispAir restatement: synthetic VM traces satisfy every transition constraint and
assertion on the trace domain; counts match ZkLispAir::new (vm/air/mod.rs:217-290)."""
import ctypes as C

import pytest


@pytest.mark.parametrize("log_n", [5, 6, 8, 10])
def test_trace_satisfies_air(oracle, log_n):
    t, pi, w = oracle.synth_segment(0x5EED0001, log_n)
    n = 1 << log_n
    rc, n_tc, n_as, ceb, ncomp = oracle.air_info(pi, w, n)
    assert rc == 0
    assert n_tc == 193            # Ctrl 91 + ALU 16 + ROM 86
    assert n_as == 141 * (n // 32) + 8   # schedule 141/level + pc + pi_prog + 6 ROM
    assert (ceb, ncomp) == (8, 7)
    assert oracle.check_trace(t, pi, w, n) == (0, 0, 0)


def test_corrupted_trace_detected(oracle):
    t, pi, w = oracle.synth_segment(0x5EED0001, 6)
    n = 64
    r_start = 42
    t[(r_start + 3) * n + 40].lo ^= 1        # register r3 at row 40 (pad rows carry)
    rc, row, idx = oracle.check_trace(t, pi, w, n)
    assert rc == 1
    opts = oracle.default_options(w, n, queries=8, grind=0)
    with pytest.raises(RuntimeError, match="degree too large"):
        oracle.prove(t, w, n, pi, opts)


def test_sponge_trace_satisfies_poseidon_block(oracle):
    """Programs with SAbsorbN / SSqueeze (features VM | SPONGE | POSEIDON): the PoseidonAir
    block (poseidon.rs:65-162: 27x12 round, 12 hold, 10 VM->lane binding constraints, first
    in evaluation order) holds on the generated trace, and corruptions inside the block's
    reach are caught by it."""
    n = 256
    t, pi, w = oracle.synth_segment(0x5EED0055, 8, 1)
    assert pi.feature_mask == 0x23 and pi.vm_usage_mask & 0x80
    assert oracle.check_trace(t, pi, w, n) == (0, 0, 0)
    # level 3 is a squeeze (cycle absorb, const, absorb, squeeze, ...): round row of round 5
    row = 3 * 32 + 1 + 5
    t[5 * n + row + 1].lo ^= 1            # lane 5 of the next state
    rc, bad_row, idx = oracle.check_trace(t, pi, w, n)
    assert rc == 1 and bad_row == row and idx < 27 * 12
    t[5 * n + row + 1].lo ^= 1
    # a map-row absorb lane that does not match the selected register: binding constraint
    lane0 = 3 * 32
    t[0 * n + lane0].lo ^= 2
    rc, bad_row, idx = oracle.check_trace(t, pi, w, n)
    assert rc == 1 and 27 * 12 + 12 <= idx < 27 * 12 + 22


def test_sponge_trace_proves_and_verifies(oracle):
    n = 1 << 7
    t, pi, w = oracle.synth_segment(0x5EED0056, 7, 1)
    opts = oracle.default_options(w, n, queries=16, grind=4)
    proof = oracle.prove(t, w, n, pi, opts)
    rc, err = oracle.verify(proof, pi, opts)
    assert rc == 0, err
