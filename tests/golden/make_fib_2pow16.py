"""Generates tests/golden/fib_2pow16.json and fib_2pow16_ops.json.gz: `zk-lisp prove
examples/fib-2pow16.zlisp` (BASELINE configs[1]'s program) pinned by the CPU oracle on a sample
of its segments.

  * the op list compile_entry emits (oracle/lower_ref.py; 458,751 ops: the loop of 2^16
    iterations unrolled, zk-lisp-compiler/src/lower/iter.rs:168-169) kept as gzip'd JSON data,
    program_id = BLAKE3(file bytes) (zk-lisp-compiler/src/lib.rs:239-245); the source text is not
    copied, only its length and BLAKE3;
  * the plan at --max-segment-rows 65536: 2^19 levels = 2^24 rows = 256 segments of 65,536 rows
    (segment_planner.rs:93-279);
  * for the sampled segments -- 0, 1, 223 (the last one with program ops: the loop's tail, End
    and the first padding level), 224 (the first all-padding segment) and 255 (the last) -- the
    oracle's per-segment trace (orc_build_segment_trace: every level streamed, no full trace;
    each checked against the oracle AIR), its sha256, the oracle's segment proof (checked by the
    oracle verifier) and zl1 step proof, and the VM state hashes.

CLI defaults: q 64, blowup 16, grind 16 (zk-lisp-cli/src/main.rs:124-132).

Run in the build container (needs /root/reference for the source; ~10 min on 8 threads):
    python tests/golden/make_fib_2pow16.py [--threads 8] [--segments 0,1,223,224,255]
"""
import argparse
import gzip
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))
import lower_ref  # noqa: E402
import oracle_lib  # noqa: E402
import segments_ref  # noqa: E402
import zkl_hip  # noqa: E402  (ZklOp / StepInfo layouts only)

OUT = os.path.join(HERE, "fib_2pow16.json")
OPS_OUT = os.path.join(HERE, "fib_2pow16_ops.json.gz")
SRC = "/root/reference/examples/fib-2pow16.zlisp"
MAX_ROWS = 1 << 16
CLI = {"queries": 64, "blowup": 16, "grind": 16, "min_security_bits": 128}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--segments", default="0,1,223,224,255")
    args = ap.parse_args()
    oracle_lib.set_threads(args.threads)
    src = open(SRC, "rb").read()
    ops_l = lower_ref.compile_entry(src.decode(), [])[0]
    pid = oracle_lib.blake3(src)
    data = json.dumps([[k, f] for k, f in ops_l], separators=(",", ":")).encode()
    with gzip.GzipFile(OPS_OUT, "wb", mtime=0) as f:
        f.write(data)
    ops = [zkl_hip.op(k, **f) for k, f in ops_l]
    arr = (zkl_hip.ZklOp * len(ops))(*ops)
    plan = segments_ref.plan_segments(len(ops), MAX_ROWS)
    print(f"fib-2pow16: {len(ops)} ops, {len(plan)} segments, program_id {pid.hex()[:16]}..", flush=True)
    res = json.load(open(OUT)) if os.path.exists(OUT) else {}
    res.update({"source": "examples/fib-2pow16.zlisp", "source_bytes": len(src), "program_id": pid.hex(),
                "n_ops": len(ops), "ops_json_sha256": sha(data), "ops_file": os.path.basename(OPS_OUT),
                "cli": CLI, "max_segment_rows": MAX_ROWS, "plan": [list(p) for p in plan]})
    segs = res.setdefault("segments", {})
    for i in [int(x) for x in args.segments.split(",")]:
        a, b = plan[i]
        t0 = time.time()
        rc, t, pi, w, sin, sout = oracle_lib.build_segment_trace(arr, pid, a, b)
        assert rc == 0, rc
        m = b - a
        assert oracle_lib.check_trace(t, pi, w, m) == (0, 0, 0), f"segment {i}: AIR rejects the trace"
        t1 = time.time()
        opts = oracle_lib.default_options(w, m, queries=CLI["queries"], blowup=CLI["blowup"], grind=CLI["grind"])
        proof = oracle_lib.prove(t, w, m, pi, opts)
        rc, err = oracle_lib.verify(proof, pi, opts)
        assert rc == 0, err
        zpi = zkl_hip.AirPublicInputs()
        zkl_hip.C.memmove(zkl_hip.C.byref(zpi), zkl_hip.C.byref(pi), zkl_hip.C.sizeof(zpi))
        info = zkl_hip.step_info_for(zpi, i, len(plan), sin, sout)
        step = oracle_lib.step_encode(pi, info, proof)
        segs[str(i)] = {"rows": [a, b], "width": w, "feature_mask": pi.segment_feature_mask,
                        "partitions": [opts.num_partitions, opts.hash_rate], "trace_sha256": sha(bytes(t)),
                        "pi_sha256": sha(bytes(pi)), "state_in": sin.hex(), "state_out": sout.hex(),
                        "proof_len": len(proof), "proof_sha256": sha(proof),
                        "step_len": len(step), "step_sha256": sha(step)}
        print(f"  segment {i} rows [{a},{b}) width {w}: trace {t1 - t0:.0f}s, proof {len(proof)} B "
              f"({time.time() - t1:.0f}s)", flush=True)
        json.dump(res, open(OUT, "w"), indent=1)
    json.dump(res, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
