"""BASELINE configs[0]: `zk-lisp prove examples/hello-zk.zlisp --arg u64:2 --arg u64:5 --secret
u64:3` (CLI defaults q 64, blowup 16, grind 16, 128-bit release target) end to end through the
library: the compiler's op list (tests/golden/hello_zk.json, derived by oracle/lower_ref.py from
the source; program_id = BLAKE3 of the file, zk-lisp-compiler/src/lib.rs:239-245), the trace
builder, the segment plan and slice, the segment proof, the zl1 step proof and the ZKLRC1
artifact the CLI writes to proof.bin (zk-lisp-cli/src/prove.rs:56-78), each pinned by the CPU
oracle's golden (tests/golden/make_hello_zk.py).  Parity against the reference itself is
unpinned (Rust; no cargo here): the goldens are the oracle restatement's bytes.
"""
import ctypes as C
import hashlib
import json
import os
import sys

import pytest

import zkl_hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
G = json.load(open(os.path.join(ROOT, "tests", "golden", "hello_zk.json")))
SRC = "/root/reference/examples/hello-zk.zlisp"


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _ops():
    return [zkl_hip.op(k, **f) for k, f in G["ops"]]


def _segments(public=None, secret=None):
    """The product's trace, plan and slices of the program: [(trace, pi, width, rows, state_in, state_out)]."""
    ops = _ops()
    t, pi, w, n = zkl_hip.build_trace(ops, bytes.fromhex(G["program_id"]),
                                      secret_args=G["cli"]["secret_u64"] if secret is None else secret,
                                      main_args=G["cli"]["public_u64"] if public is None else public)
    plan = zkl_hip.plan_segments(len(ops), G["cli"]["max_segment_rows"])
    out = []
    for a, b in plan:
        st, spi, sw, sin, sout = zkl_hip.slice_segment(t, w, n, ops, pi, a, b)
        out.append((st, spi, sw, b - a, sin, sout))
    return (t, pi, w, n), plan, out


def _opts(w, m):
    c = G["cli"]
    return zkl_hip.proof_options(w, m, queries=c["queries"], blowup=c["blowup"], grind=c["grind"])


def _step(i, total, seg, proof):
    _, spi, _, _, sin, sout = seg
    info = zkl_hip.step_info_for(spi, i, total, sin, sout, main_args=G["cli"]["public_u64"])
    return zkl_hip.step_proof_encode(spi, info, proof)


def _aggregate(steps):
    c = G["cli"]
    return zkl_hip.agg_prove(steps, queries=c["queries"], blowup=c["blowup"], grind=c["grind"],
                             min_security_bits=c["min_security_bits"])


@pytest.mark.skipif(not os.path.exists(SRC), reason="the reference tree is only in the build container")
def test_op_list_and_program_id_from_source(oracle):
    """The fixture's op list is what compile_entry lowers the file to (lower_ref restates
    lower/mod.rs, ctx.rs, operators.rs, assert.rs) and program_id is BLAKE3 of its bytes."""
    import lower_ref
    src = open(SRC, "rb").read()
    ops, schema = lower_ref.compile_entry(src.decode(), G["cli"]["public_u64"])
    assert [[k, f] for k, f in ops] == G["ops"]
    assert len(src) == G["source_bytes"] and oracle.blake3(src).hex() == G["program_id"]
    assert schema == ([("let", "u64"), ("let", "u64")], "u64")


def test_lowering_restatement_cases():
    """lower_ref on small programs whose lowering the compiler's rules fix: constant folding,
    Sethi-Ullman order, a borrowed register moved before use, the result normalised to r0."""
    import lower_ref
    ops, _ = lower_ref.compile_entry("(def (main) (+ 2 3))", [])
    assert ops == [("Const", {"dst": 7, "imm": 5}), ("Mov", {"dst": 0, "src": 7}), ("End", {})]
    ops, _ = lower_ref.compile_entry("(def (main a) (* a (+ a 1)))", [4])
    assert ops == [("Const", {"dst": 7, "imm": 20}), ("Mov", {"dst": 0, "src": 7}), ("End", {})]
    ops, _ = lower_ref.compile_entry("(def (main) (let ((s (secret-arg 1))) (- s 1)))", [])
    assert ops == [("Mov", {"dst": 7, "src": 1}), ("Const", {"dst": 6, "imm": 1}), ("Sub", {"dst": 7, "a": 7, "b": 6}),
                   ("Mov", {"dst": 0, "src": 7}), ("End", {})]
    with pytest.raises(NotImplementedError):
        lower_ref.compile_entry("(def (main) (merkle-verify 1 2))", [])
    with pytest.raises(ValueError):
        lower_ref.compile_entry("(def (main x) x)", [])


def test_trace_plan_and_oracle_chain_match_goldens(oracle):
    """The product's trace builder, planner and slicer feed the oracle prover: its segment
    proof, the product's zl1 step encoding and the product's aggregation (zkl_agg_prove) give
    the golden bytes; the product verifiers accept them."""
    (t, pi, w, n), plan, segs = _segments()
    assert (w, n) == (G["trace"]["width"], G["trace"]["rows"])
    assert [list(p) for p in plan] == [s["rows"] for s in G["segments"]]
    assert pi.n_main_slots == 2 and pi.feature_mask == zkl_hip.FM_VM
    arr = (zkl_hip.ZklOp * len(_ops()))(*_ops())
    rc, ot, _, ow, on = oracle.build_trace(arr, bytes.fromhex(G["program_id"]), secret_args=G["cli"]["secret_u64"],
                                           main_args=zkl_hip._vm_args(G["cli"]["public_u64"]))
    assert rc == 0 and bytes(ot) == bytes(t)
    steps = []
    for i, (seg, want) in enumerate(zip(segs, G["segments"])):
        st, spi, sw, m, _, _ = seg
        assert oracle.check_trace(st, spi, sw, m) == (0, 0, 0)
        o = _opts(sw, m)
        opi = oracle.AirPublicInputs()
        C.memmove(C.byref(opi), C.byref(spi), C.sizeof(opi))
        proof = oracle.prove(st, sw, m, opi, oracle.ProofOptions(*[getattr(o, f) for f, _ in o._fields_]))
        assert (len(proof), sha(proof)) == (want["proof_len"], want["proof_sha256"])
        zkl_hip.verify_segment(proof, spi, o)
        steps.append(_step(i, len(segs), seg, proof))
        assert sha(steps[-1]) == want["step_sha256"]
    art, dg = _aggregate(steps)
    assert (len(art), sha(art), dg.hex()) == (G["proof_bin"]["len"], G["proof_bin"]["sha256"],
                                             G["proof_bin"]["recursion_digest"])
    zkl_hip.agg_verify(art)


def test_wrong_secret_breaks_the_assert(oracle):
    """--secret u64:4: pub_y != pub_x + s, the Assert level's constraint fails (the reference's
    prover would emit a proof that does not verify)."""
    _, _, segs = _segments(secret=[4])
    st, spi, sw, m, _, _ = segs[0]
    rc, row, _ = oracle.check_trace(st, spi, sw, m)
    assert rc == 1


@pytest.mark.gpu
def test_hello_zk_prove_chain_on_gpu(gpu_ctx):
    """`zk-lisp prove` of configs[0] with the segment proved on the GPU: segment proof, step and
    proof.bin equal the oracle goldens; the product verifiers accept them."""
    _, _, segs = _segments()
    steps = []
    for i, (seg, want) in enumerate(zip(segs, G["segments"])):
        st, spi, sw, m, _, _ = seg
        o = _opts(sw, m)
        proof = gpu_ctx.prove_segment(st, sw, m, spi, o)
        assert (len(proof), sha(proof)) == (want["proof_len"], want["proof_sha256"])
        zkl_hip.verify_segment(proof, spi, o)
        steps.append(_step(i, len(segs), seg, proof))
    art, dg = _aggregate(steps)
    assert sha(art) == G["proof_bin"]["sha256"] and dg.hex() == G["proof_bin"]["recursion_digest"]
    zkl_hip.agg_verify(art)
