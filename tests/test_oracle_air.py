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


# generator flags: 1 sponge, 2 RAM (Load/Store), 4 Merkle path
@pytest.mark.parametrize("flags,width", [(2, 212), (4, 211), (3, 212), (5, 211), (6, 219), (7, 219)])
@pytest.mark.parametrize("log_n", [8, 11])
def test_ram_merkle_traces_satisfy_air(oracle, flags, width, log_n):
    """RamAir (ram.rs:82-236) and MerkleAir (merkle.rs:60-134) blocks, with the segment
    layouts {vm, ram, rom} = 212, {vm, merkle, rom} = 211 and the baseline 219."""
    n = 1 << log_n
    t, pi, w = oracle.synth_segment(0x5EED0300 + flags, log_n, flags)
    assert w == width
    rc, n_tc, n_as, ceb, ncomp = oracle.air_info(pi, w, n)
    assert rc == 0 and (ceb, ncomp) == (8, 7)
    n_ram = 0
    if flags & 2:
        n_ram = 7 + ((bin(pi.ram_delta_clk_bits).count("1") + 1) if pi.vm_usage_mask & 0x100 else 0)
    n_pose = 27 * 12 + 12 + (10 if flags & 1 else 0) if flags & 5 else 0
    n_sponge_sel = 40 if flags & 1 else 0
    assert n_tc == 193 + n_ram + (7 if flags & 4 else 0) + n_pose + n_sponge_sel
    assert oracle.check_trace(t, pi, w, n) == (0, 0, 0)


def test_ram_trace_uses_delta_clk_gadget(oracle):
    n = 1 << 12
    t, pi, w = oracle.synth_segment(0x5EED0001, 12, 2)
    assert pi.vm_usage_mask & 0x100 and bin(pi.ram_delta_clk_bits).count("1") >= 3
    assert oracle.check_trace(t, pi, w, n) == (0, 0, 0)


def test_ram_corruption_detected(oracle):
    """A read whose sorted-table value differs from the last write to that address."""
    n = 1 << 9
    t, pi, w = oracle.synth_segment(0x5EED0301, 9, 2)
    s_on, s_val, s_w = 149, 152, 153          # {vm, ram, rom} layout (layout.rs:247-256)
    row = next(r for r in range(n) if t[s_on * n + r].lo == 1 and t[s_w * n + r].lo == 0
               and (t[s_val * n + r].lo | t[s_val * n + r].hi))
    t[s_val * n + row].lo ^= 1
    rc, bad_row, idx = oracle.check_trace(t, pi, w, n)
    assert rc == 1


def test_merkle_root_binding(oracle):
    n = 256
    t, pi, w = oracle.synth_segment(0x99, 8, 4)
    assert pi.feature_mask == 0x43
    pi.merkle_root[0] ^= 1
    rc, bad_row, idx = oracle.check_trace(t, pi, w, n)
    assert rc == 1 and bad_row == 5 * 32 + 28      # MerkleStepLast final row


@pytest.mark.parametrize("flags", [2, 4, 7])
def test_ram_merkle_proves_and_verifies(oracle, flags):
    n = 1 << 8
    t, pi, w = oracle.synth_segment(0x5EED0400 + flags, 8, flags)
    opts = oracle.default_options(w, n, queries=16, grind=4)
    proof = oracle.prove(t, w, n, pi, opts)
    rc, err = oracle.verify(proof, pi, opts)
    assert rc == 0, err
