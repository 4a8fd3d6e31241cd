"""Generates tests/golden/hello_zk.json: BASELINE configs[0], `zk-lisp prove examples/hello-zk.zlisp
--arg u64:2 --arg u64:5 --secret u64:3` at the CLI defaults (q 64, blowup 16, grind 16,
release security 128 bits; zk-lisp-cli/src/main.rs:108-153, prove.rs:20-78), pinned by the
CPU oracle:

  * the op list compile_entry emits (oracle/lower_ref.py, a restatement of the compiler's
    lowering for the forms the program uses) and program_id = BLAKE3(file bytes)
    (zk-lisp-compiler/src/lib.rs:239-245); the file itself is not copied, only its length and
    BLAKE3 are recorded;
  * the segment plan (segment_planner.rs:93-276, default max rows 4096: one segment), the
    segment's trace width and rows, the oracle's segment proof, the zl1 step proof (with the
    typed main args 2, 5 as PublicInputs::main_args), and the ZKLRC1 artifact `prove` writes to
    proof.bin (oracle/agg_ref.py aggregation of the one step, FieldExtension::Quadratic).

Run in the build container (needs /root/reference for the source text; a few seconds):
    python tests/golden/make_hello_zk.py
"""
import ctypes as C
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))
import agg_ref  # noqa: E402
import lower_ref  # noqa: E402
import oracle_lib  # noqa: E402
import segments_ref  # noqa: E402
import zkl_hip  # noqa: E402  (ZklOp / StepInfo layouts only)

SRC = "/root/reference/examples/hello-zk.zlisp"
OUT = os.path.join(HERE, "hello_zk.json")
PUBLIC = [2, 5]   # --arg u64:2 --arg u64:5
SECRET = [3]      # --secret u64:3
MAX_SEGMENT_ROWS = 1 << 12


def chain(src_bytes, ops_list, public=PUBLIC, secret=SECRET, queries=64, blowup=16, grind=16):
    """The oracle's `zk-lisp prove` of an op list: [(segment proof, step proof)], (artifact, digest)."""
    pid = oracle_lib.blake3(src_bytes)
    ops = [zkl_hip.op(k, **f) for k, f in ops_list]
    arr = (zkl_hip.ZklOp * len(ops))(*ops)
    va = zkl_hip._vm_args(public)
    rc, t, pi, w, n = oracle_lib.build_trace(arr, pid, secret_args=secret, main_args=va)
    assert rc == 0, rc
    plan = segments_ref.plan_segments(len(ops), MAX_SEGMENT_ROWS)
    kinds = [o.kind for o in ops]
    out = []
    for i, (a, b) in enumerate(plan):
        st, spi, sw, sin, sout = segments_ref.slice_segment(oracle_lib, t, n, kinds, pi, a, b)
        m = b - a
        opts = oracle_lib.default_options(sw, m, queries=queries, blowup=blowup, grind=grind)
        proof = oracle_lib.prove(st, sw, m, spi, opts)
        rc, err = oracle_lib.verify(proof, spi, opts)
        assert rc == 0, err
        zpi = zkl_hip.AirPublicInputs()
        C.memmove(C.byref(zpi), C.byref(spi), C.sizeof(zpi))
        info = zkl_hip.step_info_for(zpi, i, len(plan), sin, sout, main_args=public)
        out.append(((a, b), sw, proof, oracle_lib.step_encode(spi, info, proof)))
    art, dg, _ = agg_ref.agg_prove(oracle_lib, [s for *_, s in out], queries=queries, blowup=blowup, grind=grind)
    return pid, w, n, plan, out, art, dg


def main():
    src = open(SRC, "rb").read()
    ops, schema = lower_ref.compile_entry(src.decode(), PUBLIC)
    assert schema == ([("let", "u64"), ("let", "u64")], "u64")  # both args are runtime public main args
    pid, w, n, plan, segs, art, dg = chain(src, ops)
    res = {
        "source": "examples/hello-zk.zlisp", "source_bytes": len(src), "program_id": pid.hex(),
        "cli": {"public_u64": PUBLIC, "secret_u64": SECRET, "queries": 64, "blowup": 16, "grind": 16,
                "min_security_bits": 128, "max_segment_rows": MAX_SEGMENT_ROWS},
        "ops": [[k, f] for k, f in ops],
        "trace": {"width": w, "rows": n},
        "segments": [{"rows": [a, b], "width": sw, "proof_len": len(p), "proof_sha256": hashlib.sha256(p).hexdigest(),
                      "step_len": len(s), "step_sha256": hashlib.sha256(s).hexdigest()} for (a, b), sw, p, s in segs],
        "proof_bin": {"len": len(art), "sha256": hashlib.sha256(art).hexdigest(), "recursion_digest": dg.hex()},
    }
    json.dump(res, open(OUT, "w"), indent=1)
    print(json.dumps(res["proof_bin"]), len(segs), "segment(s)")


if __name__ == "__main__":
    main()
