"""zl1 step proof (host code, no GPU): the library's ZKLSTP1 encoder
(StepProof::to_bytes, proof/step.rs:79-151), its decoder's root_trace (proof/format.rs:214-238)
and step digest (proof/digest.rs:16-68) against the C oracle (oracle/step.c) and an
independent pure-Python walk of the same reference code (tests/pyref.py primitives).

The inner proof is an oracle proof of a small synthetic segment; which inner proof is
wrapped does not matter to the wrapper beyond its TraceInfo, options and commitments."""
import ctypes as C
import random
import struct

import pytest

import pyref


@pytest.fixture(scope="module")
def inner(oracle):
    import zkl_hip
    t, opi, w = oracle.synth_segment(0x57E90001, 5)
    opts = oracle.default_options(w, 32, queries=8, grind=0)
    pi = zkl_hip.AirPublicInputs()  # same layout, the library's ctypes class
    C.memmove(C.byref(pi), C.byref(opi), C.sizeof(pi))
    return oracle.prove(t, w, 32, opi, opts), pi


def _info(zkl_hip, pi, seed, args=((0, 7), (1, 2**100 + 3), (2, None)), index=2, total=5):
    rng = random.Random(seed)
    info = zkl_hip.StepInfo()
    info.suite_id[:] = bytes(pi.program_id)  # prove.rs:985
    info.lambda_bits = 100
    info.segment_index, info.segments_total = index, total
    for f in ("pc_init", "state_in_hash", "state_out_hash", "ram_gp_unsorted_in", "ram_gp_unsorted_out",
              "ram_gp_sorted_in", "ram_gp_sorted_out"):
        getattr(info, f)[:] = rng.randbytes(32)
    for i in range(3):
        info.rom_s_in[i][:] = rng.randbytes(32)
        info.rom_s_out[i][:] = rng.randbytes(32)
    info.n_main_args = len(args)
    for i, (tag, v) in enumerate(args):
        info.main_args[i].tag = tag
        raw = v.to_bytes(8 if tag == 0 else 16, "little") if tag < 2 else rng.randbytes(32)
        info.main_args[i].bytes[:len(raw)] = raw
    return info


def _walk(b):
    """step.rs:153-493 field order, in Python."""
    off = 7
    assert b[:7] == b"ZKLSTP1"

    def take(k):
        nonlocal off
        off += k
        return b[off - k:off]

    d = {"lambda": struct.unpack("<I", take(4))[0], "suite": take(32), "program_id": take(32),
         "program_commitment": take(32), "merkle_root": take(32), "feature_mask": struct.unpack("<Q", take(8))[0]}
    args = []
    for _ in range(struct.unpack("<I", take(4))[0]):
        tag = take(1)[0]
        args.append((tag, take({0: 8, 1: 16, 2: 32}[tag])))
    d["args"] = args
    d["vm_usage_mask"], d["ram_delta_clk_bits"] = struct.unpack("<II", take(8))
    d["rom_acc"] = [take(32) for _ in range(3)]
    d["segment_index"], d["segments_total"] = struct.unpack("<II", take(8))
    d["pc_init"] = take(32)
    d["bnd"] = take(32 * 12)
    d["inner"] = take(struct.unpack("<I", take(4))[0])
    assert off == len(b)
    return d


def _commitments(inner):
    off = 6 + 1 + inner[6] + 10 + 1
    first = inner[off]
    ln = (first & -first).bit_length()
    enc = int.from_bytes(inner[off:off + ln], "little")
    clen = enc >> ln
    off += ln
    return inner[off:off + clen]


def _py_digest(step):
    """proof/digest.rs:16-68 over pyref (BLAKE3 RO, Poseidon suite of suite_id)."""
    d = _walk(step)
    inner = d["inner"]
    logn, blowup, q = inner[3], inner[6 + 1 + inner[6] + 1], inner[6 + 1 + inner[6]]
    idx, tot = (d["segment_index"], d["segments_total"]) if d["segments_total"] > 1 else (0, 1)
    rt = pyref.blake3(b"zkl/step/root_trace" + d["suite"] + _commitments(inner))
    slots = sum(2 if t == 2 else 1 for t, _ in d["args"])
    m = 1 << logn
    meta = struct.pack("<IHHHHIQ", m, blowup, q, 2, min(d["lambda"], 65535), 5 + slots + 13, m * q)
    pib = (d["program_id"] + d["program_commitment"] + struct.pack("<QII", d["feature_mask"], idx, tot)
           + d["pc_init"] + d["bnd"])
    S = pyref.suite(d["suite"])

    def two(l, r):
        st = [l, r] + [0] * 8 + list(S[0])
        return pyref.permute(st, S)[0]

    h_meta = two(pyref.ro("zkl/step/digest/meta", meta), 0)
    h_pi = two(pyref.ro("zkl/step/digest/pi", pib), 0)
    h_roots = two(pyref.fold32(rt), 0)
    ch = two(two(two(pyref.ro("zkl/step/digest/suite", d["suite"]), h_meta), h_pi), h_roots)
    return ch.to_bytes(16, "little") + bytes(16), rt


def test_step_encoding_matches_oracle_and_layout(oracle, inner):
    import zkl_hip
    inner_b, pi = inner
    info = _info(zkl_hip, pi, 1)
    got = zkl_hip.step_proof_encode(pi, info, inner_b)
    assert got == oracle.step_encode(pi, info, inner_b)
    d = _walk(got)
    assert d["inner"] == inner_b and d["lambda"] == 100 and d["suite"] == bytes(pi.program_id)
    assert d["feature_mask"] == pi.feature_mask and d["merkle_root"] == bytes(pi.merkle_root)
    assert (d["segment_index"], d["segments_total"]) == (2, 5)
    assert [t for t, _ in d["args"]] == [0, 1, 2]
    assert d["args"][1][1] == (2**100 + 3).to_bytes(16, "little")
    for i in range(3):
        v = pi.rom_acc[i].lo | (pi.rom_acc[i].hi << 64)
        assert d["rom_acc"][i] == v.to_bytes(16, "little") + bytes(16)  # fe_to_bytes_fold
    assert d["bnd"][:32] == bytes(info.state_in_hash) and d["bnd"][-32:] == bytes(info.rom_s_out[2])


@pytest.mark.parametrize("seed,index,total,args", [
    (1, 2, 5, ((0, 7), (1, 2**100 + 3), (2, None))),
    (2, 0, 1, ()),
    (3, 9, 0, ((2, None), (2, None))),   # total <= 1: decoded as a single-segment proof
    (4, 63, 64, ((0, 2**64 - 1),)),
])
def test_step_digest_three_ways(oracle, inner, seed, index, total, args):
    import zkl_hip
    inner_b, pi = inner
    step = zkl_hip.step_proof_encode(pi, _info(zkl_hip, pi, seed, args, index, total), inner_b)
    dg, rt = zkl_hip.step_proof_digest(step)
    assert (dg, rt) == oracle.step_digest(step)
    assert (dg, rt) == _py_digest(step)


def test_single_segment_rule(inner):
    """from_bytes rebuilds segments_total <= 1 as (0, 1) (step.rs:413-432): the digest of
    an encoding with index 5 / total 1 equals that of index 0 / total 1."""
    import zkl_hip
    inner_b, pi = inner
    a = zkl_hip.step_proof_encode(pi, _info(zkl_hip, pi, 7, (), 5, 1), inner_b)
    b = zkl_hip.step_proof_encode(pi, _info(zkl_hip, pi, 7, (), 0, 1), inner_b)
    assert a != b
    assert zkl_hip.step_proof_digest(a) == zkl_hip.step_proof_digest(b)


def test_reference_step_serialization_cases(oracle, inner):
    """The reference's own codec tests (zk-lisp-proof-winterfell/tests/step_serialization.rs):
    a to_bytes/from_bytes round trip keeps digest, state hashes, suite, meta and core pi
    (:48-106); a corrupted magic is rejected with a message naming it (:109-128); a buffer
    cut to 8 bytes (:131-149) or one byte short of its inner proof (:152-170) is rejected."""
    import zkl_hip
    inner_b, pi = inner
    info = _info(zkl_hip, pi, 11, ((0, 5), (2, None)), 0, 1)
    step = zkl_hip.step_proof_encode(pi, info, inner_b)
    d = zkl_hip.parse_step_proof(step)
    assert d["state_in_hash"] == bytes(info.state_in_hash) and d["state_out_hash"] == bytes(info.state_out_hash)
    assert d["suite_id"] == bytes(info.suite_id) and d["program_id"] == bytes(pi.program_id)
    assert d["main_args"][0] == (0, (5).to_bytes(8, "little")) and d["main_args"][1][0] == 2
    assert d["inner"] == inner_b
    assert zkl_hip.step_proof_digest(step) == _py_digest(step)
    bad = bytearray(step)
    bad[0] ^= 0xFF
    with pytest.raises(zkl_hip.ZklError, match="magic"):
        zkl_hip.step_proof_digest(bytes(bad))
    with pytest.raises(ValueError, match="magic"):
        zkl_hip.parse_step_proof(bytes(bad))
    for cut in (step[:8], step[:-1]):
        with pytest.raises(zkl_hip.ZklError, match="truncated"):
            zkl_hip.step_proof_digest(cut)
        with pytest.raises(ValueError, match="truncated"):
            oracle.step_digest(cut)
        with pytest.raises(ValueError, match="truncated"):
            zkl_hip.parse_step_proof(cut)


def _py_children_root(suite, digests, roots):
    """agg/child.rs:853-895 over pyref."""
    if not digests:
        return bytes(32)
    S = pyref.suite(suite)

    def two(l, r):
        return pyref.permute([l, r] + [0] * 8 + list(S[0]), S)[0]

    items = sorted(two(pyref.fold32(d), pyref.fold32(r)).to_bytes(16, "little") + bytes(16)
                   for d, r in zip(digests, roots))
    layer = [pyref.fold32(b) for b in items]
    while len(layer) > 1:
        layer = [two(layer[i], layer[i + 1] if i + 1 < len(layer) else layer[i]) for i in range(0, len(layer), 2)]
    return layer[0].to_bytes(16, "little") + bytes(16)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5])
def test_children_root_three_ways(oracle, n):
    import zkl_hip
    rng = random.Random(100 + n)
    suite = rng.randbytes(32)
    digests = [rng.randbytes(16) + bytes(16) for _ in range(n)]
    roots = [rng.randbytes(32) for _ in range(n)]
    got = zkl_hip.children_root(suite, digests, roots)
    assert got == oracle.children_root(suite, digests, roots) == _py_children_root(suite, digests, roots)
    if n >= 2:  # sorted leaves: the order of the children does not matter
        assert zkl_hip.children_root(suite, digests[::-1], roots[::-1]) == got


def test_step_decode_errors(oracle, inner):
    """Truncations and a bad magic / VmArg tag fail in both implementations with the
    reference's messages (step.rs:158-180, 305-309)."""
    import zkl_hip
    inner_b, pi = inner
    step = zkl_hip.step_proof_encode(pi, _info(zkl_hip, pi, 1), inner_b)
    for cut, what in ((5, "too short"), (9, "lambda_bits"), (40, "suite_id"), (143, "feature_mask"), (149, "main_args length"), (200, "VmArg"),
                      (len(step) - 10, "inner proof bytes")):
        with pytest.raises(zkl_hip.ZklError, match=what):
            zkl_hip.step_proof_digest(step[:cut])
        with pytest.raises(ValueError, match=what):
            oracle.step_digest(step[:cut])
    with pytest.raises(zkl_hip.ZklError, match="magic"):
        zkl_hip.step_proof_digest(b"ZKLSTP2" + step[7:])
    bad = bytearray(step)
    bad[7 + 4 + 128 + 8 + 4] = 9  # first VmArg tag
    with pytest.raises(zkl_hip.ZklError, match="VmArg tag"):
        zkl_hip.step_proof_digest(bytes(bad))
    info = _info(zkl_hip, pi, 1)
    info.main_args[0].tag = 3
    with pytest.raises(zkl_hip.ZklError):
        zkl_hip.step_proof_encode(pi, info, inner_b)
