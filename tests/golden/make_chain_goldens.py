"""Generates tests/golden/chain_2p16.json: the synthetic multi-segment program the bench's
configs[2]/configs[3] lines and the aggregation tests use, pinned by the CPU oracle.

One program (program seed 0x5EEDC400) cut into 64 VM-only segments of 65,536 rows (segment i
runs the ops of seed 0x5EEDC400 + i); ROM accumulator lane 0 carries from segment to segment
(rom_s_in[0] of i+1 = rom_s_out[0] of i, the chain agg/trace.rs:524-541 checks), and the zl1
VM state hashes are state_in(i) = i, state_out(i) = i + 1 (32-byte LE).  The file holds

  * rom0_in[i]: the ROM lane-0 value segment i starts from (64 entries), so each rank of a
    multi-GPU run builds only its own segments;
  * for every one of the 64 segments: length and sha256 of the oracle proof at the headline
    options (blowup 16, q 64, grind 16, partitions (4, 16)) -- BASELINE configs[3];
  * "aggregation": the aggregation of the first 8 segments (steps with segments_total 8, the
    configs[2] set): length and sha256 of the ZKLRC1 artifact and the recursion digest, from
    oracle/agg_ref.py over oracle-made step proofs (min_security_bits 128:
    FieldExtension::Quadratic; q 64, blowup 16, grind 16);
  * "aggregation_64": the same over all 64 segments (steps with segments_total 64), the
    configs[3] artifact (prove.rs:1018-1050, then lib.rs:295-551);
  * "aggregation_ref_trace": agg_ref in the reference-trace mode (agg/trace.rs:397-398 row
    count, hash_row_poseidon root errors) over the 16 first segments, whose
    trace has 16 rows like the published run's (its agg proof was 52,558 B).

  * "aggregation_64_ref_trace": the reference-trace mode over all 64 segments (64-row trace).

Proof bytes are cached per segment under .chain_cache/ (git- and gpurun-ignored) so the run can
be resumed; each proof is checked by the oracle verifier before it is used.

Run (build container, ~2-3 min per proof on 8 threads; ~2.5 h for all 64):
    python tests/golden/make_chain_goldens.py [--threads 8] [--segments 64]

Add only the aggregation entries, from proof bytes already at hand -- e.g. the GPU test's dump
(ZKL_DUMP_CHAIN=<dir> test_chain_64_segments_and_aggregation_match_goldens): every file must
hash to the committed oracle sha256 of its segment, so the inputs are the oracle's proofs:
    python tests/golden/make_chain_goldens.py --from-dir <dir>
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
import oracle_lib  # noqa: E402
import zkl_hip  # noqa: E402  (only its ctypes StepInfo layout)

OUT = os.path.join(HERE, "chain_2p16.json")
CACHE = os.environ.get("ZKL_CHAIN_CACHE", os.path.join(ROOT, ".chain_cache"))
PROGRAM = 0x5EEDC400
LOG_N = 16
SEGMENTS = 64
PINNED8 = 8
REF_TRACE_CHILDREN = 16


def steps_for(pis, proofs, total):
    out = []
    for i in range(total):
        pi = pis[i]
        zpi = zkl_hip.AirPublicInputs()
        C.memmove(C.byref(zpi), C.byref(pi), C.sizeof(zpi))
        info = zkl_hip.step_info_for(zpi, i, total, i.to_bytes(32, "little"), (i + 1).to_bytes(32, "little"))
        out.append(oracle_lib.step_encode(pi, info, proofs[i]))
    return out


def agg_entry(steps, mode=0):
    t0 = time.time()
    art, dg, _ = agg_ref.agg_prove(oracle_lib, steps, trace_mode=mode)
    print(f"aggregation of {len(steps)} (mode {mode}): {len(art)} bytes ({time.time() - t0:.0f}s)", flush=True)
    return {"children": len(steps), "queries": 64, "blowup": 16, "grind": 16, "min_security_bits": 128,
            "len": len(art), "sha256": hashlib.sha256(art).hexdigest(), "recursion_digest": dg.hex()}


def from_dir(d):
    """Aggregation entries from 64 proof files that hash to the committed segment goldens."""
    out = json.load(open(OUT))
    pis, proofs = [], []
    for i in range(SEGMENTS):
        g = out["segments"][i]
        proof = open(os.path.join(d, f"seg{i:02d}.bin"), "rb").read()
        assert g["index"] == i and hashlib.sha256(proof).hexdigest() == g["sha256"], f"segment {i} differs from its golden"
        _, pi, _ = oracle_lib.synth_segment_chain(PROGRAM, PROGRAM + i, LOG_N, int(out["rom0_in"][i], 16))
        pis.append(pi)
        proofs.append(proof)
    for key, k, mode in (("aggregation", PINNED8, 0), ("aggregation_ref_trace", REF_TRACE_CHILDREN, 1),
                         ("aggregation_64", SEGMENTS, 0), ("aggregation_64_ref_trace", SEGMENTS, 1)):
        e = agg_entry(steps_for(pis, proofs, k), mode=mode)
        if key in out:
            assert out[key] == e, f"{key}: recomputed entry differs from the committed one"
        out[key] = e
    json.dump(out, open(OUT, "w"), indent=1, sort_keys=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--segments", type=int, default=SEGMENTS)
    ap.add_argument("--skip-agg", action="store_true")
    ap.add_argument("--start", type=int, default=0, help="with --skip-agg: first segment to prove")
    ap.add_argument("--stop", type=int, default=SEGMENTS, help="with --skip-agg: one past the last segment")
    ap.add_argument("--from-dir", default=None, help="seg{i:02d}.bin proofs matching the committed hashes")
    args = ap.parse_args()
    if args.from_dir:
        return from_dir(args.from_dir)
    oracle_lib.set_threads(args.threads)
    os.makedirs(CACHE, exist_ok=True)
    n = 1 << LOG_N
    rom0, chain, pis = 0, [], []
    for i in range(SEGMENTS):
        chain.append(rom0)
        t, pi, w = oracle_lib.synth_segment_chain(PROGRAM, PROGRAM + i, LOG_N, rom0)
        pis.append(pi)
        rom0 = pi.rom_s_out[0].lo | (pi.rom_s_out[0].hi << 64)
        del t
    out = {"program_seed": PROGRAM, "log_n": LOG_N, "rom0_in": [hex(x) for x in chain], "segments": []}
    proofs = []
    for i in range(args.segments):
        if args.skip_agg and not args.start <= i < args.stop:
            continue
        path = os.path.join(CACHE, f"seg{i:02d}.bin")
        t0 = time.time()
        if os.path.exists(path):
            proof = open(path, "rb").read()
        else:
            r0 = int(chain[i], 16) if isinstance(chain[i], str) else chain[i]
            t, pi, w = oracle_lib.synth_segment_chain(PROGRAM, PROGRAM + i, LOG_N, r0)
            opts = oracle_lib.default_options(w, n)
            proof = oracle_lib.prove(t, w, n, pi, opts)
            del t
            rc, err = oracle_lib.verify(proof, pi, opts)
            assert rc == 0, err
            open(path + ".tmp", "wb").write(proof)
            os.replace(path + ".tmp", path)
        proofs.append(proof)
        out["segments"].append({"index": i, "seed": PROGRAM + i, "width": 204, "len": len(proof),
                                "sha256": hashlib.sha256(proof).hexdigest()})
        print(f"segment {i}: {len(proof)} bytes ({time.time() - t0:.0f}s)", flush=True)
    if args.skip_agg:  # proofs cached only; the golden file is left as it is
        return
    out["aggregation"] = agg_entry(steps_for(pis, proofs, PINNED8))
    if args.segments >= REF_TRACE_CHILDREN:
        out["aggregation_ref_trace"] = agg_entry(steps_for(pis, proofs, REF_TRACE_CHILDREN), mode=1)
    if args.segments >= SEGMENTS:
        out["aggregation_64"] = agg_entry(steps_for(pis, proofs, SEGMENTS))
    json.dump(out, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
