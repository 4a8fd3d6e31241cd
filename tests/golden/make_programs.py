"""Generates tests/golden/programs.json: `zk-lisp prove` of the reference's real example programs
(examples/rollup-bench.zlisp -- the published run, BASELINE configs[2]/[3]'s program -- and
examples/fib-2pow16-log-n.zlisp) pinned by the CPU oracle:

  * the op list compile_entry emits (oracle/lower_ref.py: loop/recur, if, load/store,
    safe-add/safe-sub, hash2, constant def, calls, let; zk-lisp-compiler/src/lower/*.rs) and
    program_id = BLAKE3(file bytes) (zk-lisp-compiler/src/lib.rs:239-245); the source text is not
    copied, only its length and BLAKE3;
  * for each plan -- --max-segment-rows 1024 (rollup-bench = 64 segments: BASELINE configs[3]'s
    literal workload, segment_planner.rs:108-113), the CLI default 4096 (the published rollup
    run: 16 segments) and 65536 (rollup-bench = one 65,536-row segment, the metric's shape on a
    real program) -- the segment rows and widths, the oracle's segment proofs (each
    checked by the oracle verifier), the zl1 step proofs and the ZKLRC1 aggregation artifact in
    both trace modes (agg_ref trace_mode 0 = valid, what proof.bin holds; 1 = the reference's
    trace: next_pow2(max(children, 8)) rows and hash_row_poseidon root errors, agg/trace.rs:397-398,
    553-600), with the aggregation trace's shape.

CLI arguments (zk-lisp-cli/src/main.rs:495-542): rollup-bench `--arg u64:10 --arg bytes32:0x01`
(compile_entry gets [10, 1]: a bytes32 public arg enters the compiler as its low 8 bytes LE; both
are `let` args, so PublicInputs::main_args = [U64 10, Bytes32 01 00..00]); fib-2pow16-log-n takes
no arguments.  Defaults q 64, blowup 16, grind 16, 128-bit target (Quadratic aggregation).

Run in the build container (needs /root/reference for the source text; ~10-15 min on 8 threads):
    python tests/golden/make_programs.py [--threads 8] [--only rollup-bench] [--plans 1024]
"""
import argparse
import ctypes as C
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
import agg_ref  # noqa: E402
import lower_ref  # noqa: E402
import oracle_lib  # noqa: E402
import segments_ref  # noqa: E402
import zkl_hip  # noqa: E402  (ZklOp / StepInfo / VmArg layouts only)

OUT = os.path.join(HERE, "programs.json")
EXAMPLES = "/root/reference/examples"
PROGRAMS = {
    # name: (compile_entry u64 args, PublicInputs::main_args as zkl_vm_arg (tag, bytes), secrets)
    "rollup-bench": ([10, 1], [(0, (10).to_bytes(8, "little")), (2, bytes([1]))], []),
    "fib-2pow16-log-n": ([], [], []),
}
PLANS = [1 << 10, 1 << 12, 1 << 16]
CLI = {"queries": 64, "blowup": 16, "grind": 16, "min_security_bits": 128}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def prove_plan(pid, ops_list, main_args, secret, max_rows, log=print):
    """The oracle's `zk-lisp prove` of an op list under one plan."""
    ops = [zkl_hip.op(k, **f) for k, f in ops_list]
    arr = (zkl_hip.ZklOp * len(ops))(*ops)
    va = zkl_hip._vm_args(main_args) if main_args else None  # a 1-entry array would add a zero arg
    rc, t, pi, w, n = oracle_lib.build_trace(arr, pid, secret_args=secret, main_args=va)
    assert rc == 0, rc
    plan = segments_ref.plan_segments(len(ops), max_rows)
    kinds = [o.kind for o in ops]
    segs, steps = [], []
    for i, (a, b) in enumerate(plan):
        t0 = time.time()
        st, spi, sw, sin, sout = segments_ref.slice_segment(oracle_lib, t, n, kinds, pi, a, b)
        m = b - a
        assert oracle_lib.check_trace(st, spi, sw, m) == (0, 0, 0), f"segment {i}: AIR rejects the slice"
        opts = oracle_lib.default_options(sw, m, queries=CLI["queries"], blowup=CLI["blowup"], grind=CLI["grind"])
        proof = oracle_lib.prove(st, sw, m, spi, opts)
        rc, err = oracle_lib.verify(proof, spi, opts)
        assert rc == 0, err
        zpi = zkl_hip.AirPublicInputs()
        C.memmove(C.byref(zpi), C.byref(spi), C.sizeof(zpi))
        info = zkl_hip.step_info_for(zpi, i, len(plan), sin, sout, main_args=main_args)
        step = oracle_lib.step_encode(spi, info, proof)
        steps.append(step)
        segs.append({"rows": [a, b], "width": sw, "feature_mask": spi.segment_feature_mask,
                     "partitions": [opts.num_partitions, opts.hash_rate],
                     "proof_len": len(proof), "proof_sha256": sha(proof),
                     "step_len": len(step), "step_sha256": sha(step)})
        log(f"  segment {i} rows [{a},{b}) width {sw}: {len(proof)} B ({time.time() - t0:.1f}s)")
        del st
    aggs = {}
    for mode, key in ((0, "valid"), (1, "reference_trace")):
        t0 = time.time()
        try:
            art, dg, T = agg_ref.agg_prove(oracle_lib, steps, queries=CLI["queries"], blowup=CLI["blowup"],
                                           grind=CLI["grind"], min_security_bits=CLI["min_security_bits"],
                                           trace_mode=mode)
        except AssertionError as e:
            # the valid mode refuses a batch whose trace violates ZlAggAir: rollup-bench
            # at 1024 rows cuts its sorted RAM table, and the sorted grand product at a segment's last
            # row (ram_gp_sorted_out, prove.rs:1224-1227) misses the sorted row there that the next
            # segment's first row already counts (agg/trace.rs:515-521 chains out -> in)
            aggs[key] = {"rejected": str(e)}
            log(f"  aggregation ({key}): rejected: {e}")
            continue
        aggs[key] = {"len": len(art), "sha256": sha(art), "recursion_digest": dg.hex(),
                     "trace_width": len(T), "trace_rows": len(T[0])}
        log(f"  aggregation ({key}): {len(art)} B, trace {len(T)} cols x {len(T[0])} rows ({time.time() - t0:.0f}s)")
    return {"max_segment_rows": max_rows, "trace": {"width": w, "rows": n}, "segments": segs, "aggregation": aggs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--only", default=None)
    ap.add_argument("--plans", default=None, help="comma-separated max segment rows (default: all); others kept")
    args = ap.parse_args()
    oracle_lib.set_threads(args.threads)
    res = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name, (u64_args, main_args, secret) in PROGRAMS.items():
        if args.only and name != args.only:
            continue
        src = open(os.path.join(EXAMPLES, name + ".zlisp"), "rb").read()
        ops, schema, blocks = lower_ref.compile_entry(src.decode(), u64_args, with_blocks=True)
        pid = oracle_lib.blake3(src)
        print(f"{name}: {len(ops)} ops, program_id {pid.hex()[:16]}..", flush=True)
        entry = {"source": f"examples/{name}.zlisp", "source_bytes": len(src), "program_id": pid.hex(),
                 "cli": dict(CLI, compile_args=u64_args, main_args=[[tg, bytes(b).hex()] for tg, b in main_args],
                             secret_u64=secret),
                 "schema": [[list(a) for a in schema[0]], schema[1]] if schema else None,
                 "ops": [[k, f] for k, f in ops], "blocks": [list(b) for b in blocks],
                 "plans": dict(res.get(name, {}).get("plans", {}))}
        for mr in ([int(x) for x in args.plans.split(",")] if args.plans else PLANS):
            print(f" plan max_segment_rows {mr}", flush=True)
            entry["plans"][str(mr)] = prove_plan(pid, ops, main_args, secret, mr,
                                                 log=lambda s: print(s, flush=True))
        res[name] = entry
        json.dump(res, open(OUT, "w"), indent=1)
    json.dump(res, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
