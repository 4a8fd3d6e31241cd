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
