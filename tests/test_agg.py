"""Aggregation proof (host code, no GPU): the library's zkl_agg_prove /
zkl_agg_trace (build_public lib.rs:404-482, RecursionBackend::prove lib.rs:295-344 ->
prove_agg_proof prove.rs:629-719, ZKLRC1 lib.rs:486-551) against oracle/agg_ref.py, an
independent Python restatement over the C oracle's hashing.

Children are oracle proofs of small synthetic segments of one program whose ROM lane 0 and
VM state hashes chain from segment to segment (the chains agg/trace.rs:443-655 checks)."""
import ctypes as C
import hashlib
import os
import struct
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import agg_ref  # noqa: E402
import pyref  # noqa: E402

PROGRAM = 0x5EEDA900


def _steps(oracle, zkl_hip, count, log_n=5, flags=0, program=PROGRAM, break_chain_at=None, queries=8, grind=4,
           partitions=None):
    """count chained segments -> oracle proofs -> zl1 steps (the library's encoder; test_step pins it).
    partitions: force ProofOptions' num_partitions (with >= 2 the composition rows are one chunk
    narrower than the partition, where the row-digest rules of DESIGN.md §3.1 differ)."""
    n = 1 << log_n
    rom0, out = 0, []
    for i in range(count):
        t, pi, w = oracle.synth_segment_chain(program, program + i, log_n, rom0 if i != break_chain_at else rom0 + 1,
                                              flags)
        opts = oracle.default_options(w, n, queries=queries, grind=grind)
        if partitions:
            opts.num_partitions = partitions
        proof = oracle.prove(t, w, n, pi, opts)
        zpi = zkl_hip.AirPublicInputs()
        C.memmove(C.byref(zpi), C.byref(pi), C.sizeof(zpi))
        info = zkl_hip.step_info_for(zpi, i, count, i.to_bytes(32, "little"), (i + 1).to_bytes(32, "little"))
        out.append(zkl_hip.step_proof_encode(zpi, info, proof))
        rom0 = pi.rom_s_out[0].lo | (pi.rom_s_out[0].hi << 64)
    return out


@pytest.fixture(scope="module")
def z():
    import zkl_hip
    return zkl_hip


@pytest.fixture(scope="module")
def chain3(oracle, z):
    return _steps(oracle, z, 3)


@pytest.mark.parametrize("count", [1, 3])
def test_aggregation_matches_oracle(oracle, z, count, chain3):
    steps = chain3 if count == 3 else _steps(oracle, z, 1, program=PROGRAM + 0x100)
    art, dg = z.agg_prove(steps, queries=64, blowup=16, grind=8)
    want_art, want_dg, want_T = agg_ref.agg_prove(oracle, steps, queries=64, blowup=16, grind=8)
    assert z.agg_trace(steps) == want_T
    assert dg == want_dg
    assert art == want_art


def test_aggregation_default_options_quadratic(oracle, z, chain3):
    """CLI defaults (q 64, blowup 16, grind 16, 128-bit target -> FieldExtension::Quadratic)."""
    art, dg = z.agg_prove(chain3)
    want_art, want_dg, _ = agg_ref.agg_prove(oracle, chain3)
    assert art == want_art and dg == want_dg
    proof = z.parse_agg_artifact(art)["proof"]
    assert proof[6 + 1 + 16 + 3] == 2  # ProofOptions field_extension byte: Quadratic
    # extension elements are 32 bytes: the OOD frame (2 x (31 + 2) elements) is twice as long as
    # in a base-field proof of the same trace
    base, _ = z.agg_prove(chain3, min_security_bits=64)
    assert z.parse_agg_artifact(base)["proof"][6 + 1 + 16 + 3] == 1
    assert len(proof) > len(z.parse_agg_artifact(base)["proof"])


def test_aggregation_base_field_below_128_bits(oracle, z, chain3):
    art, dg = z.agg_prove(chain3, queries=64, blowup=16, grind=8, min_security_bits=64)
    want_art, want_dg, _ = agg_ref.agg_prove(oracle, chain3, queries=64, blowup=16, grind=8, min_security_bits=64)
    assert art == want_art and dg == want_dg


@pytest.mark.parametrize("flags,log_n", [(2, 6), (1, 6)])
def test_aggregation_other_layouts(oracle, z, flags, log_n):
    """Children in the {vm, ram, rom} (W 212) and sponge segment layouts."""
    steps = _steps(oracle, z, 2, log_n=log_n, flags=flags, program=PROGRAM + 0x200 + flags)
    art, dg = z.agg_prove(steps, grind=8)
    want_art, want_dg, _ = agg_ref.agg_prove(oracle, steps, grind=8)
    assert art == want_art and dg == want_dg


def test_power_of_two_children_keep_a_padding_row(oracle, z):
    """8 children: the reference's next_pow2(max(8, 8)) = 8 rows would put the last child's
    pre-increment accumulators on the asserted last row (agg/air.rs:276-304); the trace keeps
    one padding row (16 rows) and the batch proves and verifies."""
    steps = _steps(oracle, z, 8, program=PROGRAM + 0x500, queries=4, grind=0)
    T = z.agg_trace(steps)
    assert len(T[0]) == 16 and T[agg_ref.VACC][-1] == 8 * 32 * 4 and T[agg_ref.CNT][-1] == 8
    art, dg = z.agg_prove(steps, grind=8)
    want_art, want_dg, _ = agg_ref.agg_prove(oracle, steps, grind=8)
    assert art == want_art and dg == want_dg
    z.agg_verify(art)


@pytest.mark.parametrize("count", [3, 8])
def test_reference_trace_mode_matches_restatement(oracle, z, count):
    """ZKL_AGG_TRACE_REFERENCE: the trace agg/trace.rs:397-398,553-690 builds -- next_pow2(max(
    children, 8)) rows, root errors from hash_row_poseidon leaves (agg/child.rs:1025-1045) --
    equals agg_ref's reference mode cell for cell, and so does the artifact.  Children proved
    with 2 partitions: their composition rows (C < 16 columns) are one chunk, which the
    reference hashes without the merge, so every path it rebuilds ends on another root and the
    constraint root error is num_queries x (that root - the committed root); the trace rows
    (two chunks) give zero."""
    steps = _steps(oracle, z, count, program=PROGRAM + 0x600 + count, queries=4, grind=0, partitions=2)
    T1 = z.agg_trace(steps, z.AGG_TRACE_REFERENCE)
    art, dg = z.agg_prove(steps, grind=8, trace_mode=z.AGG_TRACE_REFERENCE)
    want_art, want_dg, want_T = agg_ref.agg_prove(oracle, steps, grind=8, trace_mode=1)
    assert T1 == want_T
    assert art == want_art and dg == want_dg
    assert len(T1[0]) == 8  # no padding row for 8 children
    T0 = z.agg_trace(steps)
    assert len(T0[0]) == (16 if count == 8 else 8)
    assert set(T1[agg_ref.TRE]) == {0} and set(T0[agg_ref.CRE]) == {0}
    assert all(T1[agg_ref.CRE][i] != 0 for i in range(count)) and set(T1[agg_ref.CRE][count:]) <= {0}
    # the reference's release prover proves this trace; it does not verify (C3 != 0, and with 8
    # children also v_units_acc[last]); the valid mode's artifact does
    with pytest.raises(z.ZklError):
        z.agg_verify(art)
    z.agg_verify(z.agg_prove(steps, grind=8)[0])


def test_reference_trace_mode_single_chunk_rows_agree(oracle, z, chain3):
    """With one partition (rows below 2^14) the two row-digest rules coincide: the reference
    mode's root errors are zero and, below 8 children, its trace is the valid mode's."""
    assert z.agg_trace(chain3, z.AGG_TRACE_REFERENCE) == z.agg_trace(chain3)
    art1, _ = z.agg_prove(chain3, grind=8, trace_mode=z.AGG_TRACE_REFERENCE)
    assert art1 == z.agg_prove(chain3, grind=8)[0]


def test_aggregation_trace_layout(oracle, z, chain3):
    """AggColumns (agg/layout.rs:97-175) on an honest batch: one seg_first row per child,
    accumulators before the increment, zero error columns, the FRI sample satisfies C12/C13."""
    T = z.agg_trace(chain3)
    P = agg_ref.P
    rows = len(T[0])
    assert rows == 8
    assert T[agg_ref.SEG] == [1, 1, 1] + [0] * 5
    v = 32 * 8  # m * q of each child
    assert T[agg_ref.VCH][:3] == [v] * 3 and T[agg_ref.VACC] == [0, v, 2 * v] + [3 * v] * 5
    assert T[agg_ref.CNT] == [0, 1, 2] + [3] * 5
    for col in (agg_ref.OK, agg_ref.TRE, agg_ref.CRE, agg_ref.COMP, agg_ref.ADZ, agg_ref.ML0, agg_ref.FLL,
                agg_ref.VMERR, agg_ref.RUERR, agg_ref.RSERR, agg_ref.RO0, agg_ref.RO1, agg_ref.RO2):
        assert set(T[col]) == {0}, col
    for r in range(3):
        c = [T[k][r] for k in range(agg_ref.NCOLS)]
        assert c[agg_ref.FVN] == c[agg_ref.FQ1]
        assert (c[agg_ref.FVN] * (c[agg_ref.FX1] - c[agg_ref.FX0]) -
                (c[agg_ref.FV1] * (c[agg_ref.FAL] - c[agg_ref.FX0]) - c[agg_ref.FV0] * (c[agg_ref.FAL] - c[agg_ref.FX1]))) % P == 0


def test_artifact_fields_and_digest(oracle, z, chain3):
    """ZKLRC1 fields (lib.rs:486-551) and recursion_digest_from_agg_pi (prove.rs:585-616)
    recomputed here from the step proofs with pyref's BLAKE3."""
    art, dg = z.agg_prove(chain3, grind=8)
    d = z.parse_agg_artifact(art)
    steps = [z.parse_step_proof(s) for s in chain3]
    assert d["children_count"] == 3 and d["children_ms"] == [32] * 3
    assert d["v_units_total"] == 3 * 32 * 8 and (d["m"], d["rho"], d["q"], d["o"]) == (32, 16, 8, 2)
    assert d["suite_id"] == steps[0]["suite_id"] and d["batch_id"] == bytes(32)
    assert d["vm_state_initial"] == (0).to_bytes(32, "little") and d["vm_state_final"] == (3).to_bytes(32, "little")
    assert d["rom_s_initial"] == steps[0]["rom_s_in"] and d["rom_s_final"] == steps[-1]["rom_s_out"]
    dig = [z.step_proof_digest(s) for s in chain3]
    assert d["children_root"] == z.children_root(steps[0]["suite_id"], [a for a, _ in dig], [b for _, b in dig])
    pi = b"zkl/pi/v1" + steps[0]["program_id"] + steps[0]["program_commitment"] + steps[0]["merkle_root"]
    pi += struct.pack("<QI", steps[0]["feature_mask"], len(steps[0]["main_args"]))
    assert d["pi_digest"] == pyref.blake3(pi)
    rd = (b"zkl/recursion/agg" + d["suite_id"] + d["batch_id"] + d["children_root"] +
          struct.pack("<IQ", d["children_count"], d["v_units_total"]) +
          struct.pack("<IHHHHIQ", d["m"], d["rho"], d["q"], d["o"], d["lambda"], d["pi_len"], d["v_units"]) +
          struct.pack("<IBBB", d["lde_blowup"], d["folding_factor"], d["redundancy"], d["num_layers"]) +
          struct.pack("<HI", d["num_queries"], d["grinding_factor"]))
    assert dg == pyref.blake3(rd)


def test_aggregation_rejections(oracle, z, chain3):
    with pytest.raises(z.ZklError, match="at least one step"):
        z.agg_prove([])
    # a child whose inner proof was tampered with does not replay (agg/fs.rs:38-245 + openings)
    bad = bytearray(chain3[1])
    bad[-200] ^= 1
    with pytest.raises(z.ZklError, match="does not replay|truncated|invalid"):
        z.agg_prove([chain3[0], bytes(bad), chain3[2]], grind=8)
    # ROM lane 0 not carried from segment 0 to 1: the chain error column is non-zero and the
    # trace does not satisfy ZlAggAir (the reference's prover fails the same way)
    broken = _steps(oracle, z, 2, program=PROGRAM + 0x300, break_chain_at=1)
    T = z.agg_trace(broken)
    assert T[agg_ref.RO0][1] != 0
    with pytest.raises(z.ZklError, match="does not satisfy ZlAggAir"):
        z.agg_prove(broken, grind=8)
    # steps of two different programs
    other = _steps(oracle, z, 1, program=PROGRAM + 0x400)
    with pytest.raises(z.ZklError, match="suite_id|program_id"):
        z.agg_prove([chain3[0], other[0]], grind=8)
    # an incomplete segment chain (segments_total 3, two children)
    with pytest.raises(z.ZklError, match="contiguous segment chain"):
        z.agg_prove(chain3[:2], grind=8)
    # options below the requested 128-bit conjectured security (prove.rs:664-681)
    with pytest.raises(z.ZklError, match="min_security_bits"):
        z.agg_prove(chain3, queries=16, blowup=8, grind=0)
    # winterfell's ProofOptions::new bound: grinding factor <= 32 (a grind > 64 could never be met)
    with pytest.raises(z.ZklError, match="grinding factor"):
        z.agg_prove(chain3, grind=33)
    with pytest.raises(z.ZklError, match="trace mode"):
        z.agg_prove(chain3, grind=8, trace_mode=2)


def test_artifact_hash_is_stable(oracle, z, chain3):
    """Determinism: two runs give the same artifact (the grinding search is multi-threaded,
    the nonce it returns is the minimum, as winterfell's sequential search)."""
    a1, _ = z.agg_prove(chain3, grind=12)
    a2, _ = z.agg_prove(chain3, grind=12)
    assert hashlib.sha256(a1).digest() == hashlib.sha256(a2).digest()


@pytest.mark.parametrize("bits", [128, 64])
def test_agg_verifier_accepts_and_rejects(oracle, z, chain3, bits):
    """zkl_agg_verify (verify_agg_proof, prove.rs:732-791): the library's artifact verifies;
    a flipped byte anywhere in the proof, a changed public input, or a security target above
    what the options give is rejected."""
    art, _ = z.agg_prove(chain3, grind=8, min_security_bits=bits)
    z.agg_verify(art, bits)
    d = z.parse_agg_artifact(art)
    head = len(art) - len(d["proof"])
    import random
    rng = random.Random(bits)
    for off in sorted(rng.sample(range(head + 40, len(art)), 12)):
        bad = bytearray(art)
        bad[off] ^= 1 << rng.randrange(8)
        with pytest.raises(z.ZklError):
            z.agg_verify(bytes(bad), bits)
    # public inputs: v_units_total (asserted at the last row) and the children root (in the seed)
    for field_off in (6 + 5 * 32, 6 + 3 * 32):
        bad = bytearray(art)
        bad[field_off] ^= 1
        with pytest.raises(z.ZklError):
            z.agg_verify(bytes(bad), bits)
    with pytest.raises(z.ZklError, match="conjectured security"):
        z.agg_verify(art, 200)
    with pytest.raises(z.ZklError, match="magic"):
        z.agg_verify(b"ZKLRC0" + art[6:], bits)
    with pytest.raises(z.ZklError, match="truncated"):
        z.agg_verify(art[:-9], bits)


def test_agg_verifier_accepts_oracle_artifact(oracle, z, chain3):
    want_art, _, _ = agg_ref.agg_prove(oracle, chain3, grind=8)
    z.agg_verify(want_art)
