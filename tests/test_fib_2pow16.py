"""examples/fib-2pow16.zlisp -- the program BASELINE configs[1] names -- end to end.

The loop of 2^16 iterations is unrolled by the compiler (lower/iter.rs:168-169): 458,751 ops,
2^19 levels, 2^24 rows, i.e. 256 segments of 65,536 rows at --max-segment-rows 65536
(segment_planner.rs:93-279).  The full trace (~55 GB at 204 columns) is never built: the product's
per-segment builder (zkl_program_new / zkl_build_segment_trace) writes each segment from a
one-pass run of the program, and its oracle twin (orc_build_segment_trace) streams every level
through a 32-row scratch.  tests/golden/fib_2pow16.json (make_fib_2pow16.py) holds the oracle's
traces, proofs and zl1 steps of segments 0, 1, 223 (the loop's tail, End and the first padding
level), 224 (the first all-padding segment) and 255; tests/golden/fib_2pow16_ops.json.gz the op
list (data: the compiler's output, lowered by oracle/lower_ref.py).
"""
import ctypes as C
import gzip
import hashlib
import json
import os
import sys
import threading

import pytest

import zkl_hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GDIR = os.path.join(ROOT, "tests", "golden")
G = json.load(open(os.path.join(GDIR, "fib_2pow16.json")))
SRC = "/root/reference/examples/fib-2pow16.zlisp"
have_ref = pytest.mark.skipif(not os.path.exists(SRC), reason="the reference tree is only in the build container")

_cache = {}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def ops_list():
    if "ops" not in _cache:
        raw = gzip.open(os.path.join(GDIR, G["ops_file"])).read()
        assert sha(raw) == G["ops_json_sha256"]
        _cache["ops"] = json.loads(raw)
    return _cache["ops"]


def program():
    if "prog" not in _cache:
        ops = [zkl_hip.op(k, **f) for k, f in ops_list()]
        _cache["zops"] = ops
        _cache["prog"] = zkl_hip.Program(ops, bytes.fromhex(G["program_id"]))
    return _cache["prog"]


# ------------------------------------------------------------------ CPU
@have_ref
def test_op_list_fixture_is_the_compilers_output(oracle):
    """The committed op list is what compile_entry lowers examples/fib-2pow16.zlisp to, and
    program_id is BLAKE3 of the file."""
    import lower_ref
    src = open(SRC, "rb").read()
    ops = lower_ref.compile_entry(src.decode(), [])[0]
    assert [[k, f] for k, f in ops] == ops_list()
    assert len(src) == G["source_bytes"] and oracle.blake3(src).hex() == G["program_id"]


def test_plan_is_256_segments_of_65536_rows():
    ops = ops_list()
    assert len(ops) == G["n_ops"] == 458751 and ops[-1][0] == "End"
    plan = zkl_hip.plan_segments(len(ops), G["max_segment_rows"])
    assert [list(p) for p in plan] == G["plan"]
    assert len(plan) == 256 and all(b - a == 1 << 16 for a, b in plan)
    P = program()
    assert (P.width, P.n_rows) == (204, 1 << 24)


@pytest.mark.parametrize("i", sorted(int(k) for k in G["segments"]))
def test_segment_trace_matches_oracle_golden(i):
    """The product's segment trace, AIR public inputs and VM state hashes equal the oracle's
    (sha256 of the bytes the oracle's streaming builder produced)."""
    g = G["segments"][str(i)]
    a, b = g["rows"]
    t, pi, w, sin, sout = program().segment(a, b)
    assert (w, pi.segment_feature_mask) == (g["width"], g["feature_mask"])
    assert sha(bytes(t)) == g["trace_sha256"] and sha(bytes(pi)) == g["pi_sha256"]
    assert (sin.hex(), sout.hex()) == (g["state_in"], g["state_out"])


def test_segment_chain_boundaries():
    """Consecutive segments chain: ROM lane 0, the VM state hash and pc run on from one segment
    into the next (what the aggregation checks, agg/trace.rs:524-541)."""
    P = program()
    prev = None
    for i in (0, 1, 2, 222, 223, 224, 225):
        t, pi, w, sin, sout = P.segment(i << 16, (i + 1) << 16)
        assert pi.pc_init.lo == i << 11
        if prev is not None and prev[0] == i - 1:
            assert (prev[1].rom_s_out[0].lo, prev[1].rom_s_out[0].hi) == (pi.rom_s_in[0].lo, pi.rom_s_in[0].hi)
            assert prev[2] == sin
        prev = (i, pi, sout)


def test_oracle_twin_equals_product_on_a_padding_segment(oracle):
    """orc_build_segment_trace (every level streamed through a scratch) gives the product's bytes
    on segment 230 (no golden proof: the trace alone)."""
    ops = [zkl_hip.op(k, **f) for k, f in ops_list()]
    arr = (zkl_hip.ZklOp * len(ops))(*ops)
    a, b = 230 << 16, 231 << 16
    rc, ot, opi, ow, oin, oout = oracle.build_segment_trace(arr, bytes.fromhex(G["program_id"]), a, b)
    t, pi, w, sin, sout = program().segment(a, b)
    assert rc == 0 and ow == w and bytes(ot) == bytes(t) and bytes(opi) == bytes(pi) and (oin, oout) == (sin, sout)


# ------------------------------------------------------------------ GPU: all 256 segments
@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_all_256_segments_prove_verify_and_aggregate_on_gpu():
    """`zk-lisp prove examples/fib-2pow16.zlisp --max-segment-rows 65536`: all 256 segments built
    by the per-segment builder into pinned trace buffers and proved on the GPU with 4 contexts in
    flight (zkl_hip.program.prove_program); the sampled segments' proofs and zl1 steps equal the
    oracle goldens; the product verifier accepts every proof; the 256 steps aggregate in the
    valid trace mode (artifact verified) and in the reference trace mode (256-row trace)."""
    from zkl_hip.program import prove_program, steps_of
    P = program()
    plan = [tuple(p) for p in G["plan"]]
    recs = prove_program(P, plan, inflight=4, builders=8)
    assert sorted(recs) == list(range(256))
    for k, g in G["segments"].items():
        r = recs[int(k)]
        assert (len(r.proof), sha(r.proof)) == (g["proof_len"], g["proof_sha256"]), f"segment {k}"
    errs = []

    def verify(part):
        for r in part:
            try:
                zkl_hip.verify_segment(r.proof, r.pi, r.opts)
            except Exception as e:  # noqa: BLE001
                errs.append((r.index, str(e)))

    rs = [recs[i] for i in range(256)]
    th = [threading.Thread(target=verify, args=(rs[k::8],)) for k in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs[:3]
    steps = steps_of(rs, 256)
    for k, g in G["segments"].items():
        assert sha(steps[int(k)]) == g["step_sha256"], f"step {k}"
    c = G["cli"]
    art, dg = zkl_hip.agg_prove(steps, queries=c["queries"], blowup=c["blowup"], grind=c["grind"],
                                min_security_bits=c["min_security_bits"])
    zkl_hip.agg_verify(art)
    assert len(zkl_hip.agg_trace(steps)[0]) == 512  # next_pow2(max(256 + 1, 8)): one padding row
    ref, _ = zkl_hip.agg_prove(steps, queries=c["queries"], blowup=c["blowup"], grind=c["grind"],
                               min_security_bits=c["min_security_bits"], trace_mode=zkl_hip.AGG_TRACE_REFERENCE)
    assert len(ref) > 0
    assert len(zkl_hip.agg_trace(steps, trace_mode=zkl_hip.AGG_TRACE_REFERENCE)[0]) == 256
