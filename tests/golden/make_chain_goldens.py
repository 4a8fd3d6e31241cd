"""Generates tests/golden/chain_2p16.json: the synthetic multi-segment program the bench's
configs[2]/configs[3] lines and the aggregation tests use, pinned by the CPU oracle.

One program (program seed 0x5EEDC400) cut into 64 VM-only segments of 65,536 rows (segment i
runs the ops of seed 0x5EEDC400 + i); ROM accumulator lane 0 carries from segment to segment
(rom_s_in[0] of i+1 = rom_s_out[0] of i, the chain agg/trace.rs:524-541 checks), and the zl1
VM state hashes are state_in(i) = i, state_out(i) = i + 1 (32-byte LE).  The file holds

  * rom0_in[i]: the ROM lane-0 value segment i starts from (64 entries), so each rank of a
    multi-GPU run builds only its own segments;
  * for the first 8 segments: length and sha256 of the oracle proof at the headline options
    (blowup 16, q 64, grind 16, partitions (4, 16));
  * the aggregation of those 8 segments: length and sha256 of the ZKLRC1 artifact and the
    recursion digest, from oracle/agg_ref.py over oracle-made step proofs (min_security_bits
    128: FieldExtension::Quadratic; q 64, blowup 16, grind 16).

Run (build container, ~2-3 min per proof on 8 threads):
    python tests/golden/make_chain_goldens.py [--threads 8]
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
PROGRAM = 0x5EEDC400
LOG_N = 16
SEGMENTS = 64
PINNED = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    args = ap.parse_args()
    oracle_lib.set_threads(args.threads)
    n = 1 << LOG_N
    rom0, chain = 0, []
    pis = []
    for i in range(SEGMENTS):
        chain.append(rom0)
        t, pi, w = oracle_lib.synth_segment_chain(PROGRAM, PROGRAM + i, LOG_N, rom0)
        if i < PINNED:
            pis.append((t, pi, w))
        rom0 = pi.rom_s_out[0].lo | (pi.rom_s_out[0].hi << 64)
    out = {"program_seed": PROGRAM, "log_n": LOG_N, "rom0_in": [hex(x) for x in chain], "segments": []}
    steps = []
    for i, (t, pi, w) in enumerate(pis):
        opts = oracle_lib.default_options(w, n)
        t0 = time.time()
        proof = oracle_lib.prove(t, w, n, pi, opts)
        rc, err = oracle_lib.verify(proof, pi, opts)
        assert rc == 0, err
        out["segments"].append({"index": i, "seed": PROGRAM + i, "width": w, "len": len(proof),
                                "sha256": hashlib.sha256(proof).hexdigest()})
        zpi = zkl_hip.AirPublicInputs()
        C.memmove(C.byref(zpi), C.byref(pi), C.sizeof(zpi))
        info = zkl_hip.step_info_for(zpi, i, PINNED, i.to_bytes(32, "little"), (i + 1).to_bytes(32, "little"))
        steps.append(oracle_lib.step_encode(pi, info, proof))
        print(f"segment {i}: {len(proof)} bytes ({time.time() - t0:.0f}s)", flush=True)
    art, dg, _ = agg_ref.agg_prove(oracle_lib, steps)
    out["aggregation"] = {"children": PINNED, "queries": 64, "blowup": 16, "grind": 16, "min_security_bits": 128,
                          "len": len(art), "sha256": hashlib.sha256(art).hexdigest(), "recursion_digest": dg.hex()}
    json.dump(out, open(OUT, "w"), indent=1, sort_keys=True)
    print(json.dumps(out["aggregation"]))


if __name__ == "__main__":
    main()
