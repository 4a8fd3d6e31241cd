"""Generates tests/golden/proof_2p16.json: length and sha256 of the CPU oracle's proof bytes
at the BASELINE headline configuration (configs[1]: 65,536 rows, blowup 16, q 64, grind 16,
partitions (4, 16) — select_partitions_for_trace, utils.rs:394-409), for

  * the eight VM-only segments of configs[2] / the bench ranks (seeds 0x5EED0001..8, W 204),
  * a sponge segment (Poseidon AIR block on, seed 0x5B0A6E10, W 204),
  * a sponge + RAM + Merkle segment (baseline layout W 219, seed 0x5EED0700).

The proofs come from oracle/ (the C restatement; "parity unpinned" at the Winterfell
boundary) with the default row-digest rule (Winterfell commit_to_rows,
DESIGN.md §3.1).  Every case exercises the 4-partition trace row digest (4 x 51 columns +
merge_many) and the one-chunk composition row digest (7 columns < partition size 16).
The GPU tests (tests/test_gpu_parity.py::test_headline_*) and bench.py compare against it.

Run (build container, ~2-3 min per proof on 8 threads):
    python tests/golden/make_proof_goldens.py [--threads 8] [--only NAME ...]
"""
import argparse
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib  # noqa: E402

OUT = os.path.join(HERE, "proof_2p16.json")
LOG_N = 16

CASES = {f"vm_{i}": (0x5EED0000 + i, 0) for i in range(1, 9)}
CASES["sponge"] = (0x5B0A6E10, 1)
CASES["sponge_ram_merkle"] = (0x5EED0700, 7)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    oracle_lib.set_threads(args.threads)
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    n = 1 << LOG_N
    for name, (seed, flags) in CASES.items():
        if args.only and name not in args.only:
            continue
        t, pi, w = oracle_lib.synth_segment(seed, LOG_N, flags)
        opts = oracle_lib.default_options(w, n)
        t0 = time.time()
        proof = oracle_lib.prove(t, w, n, pi, opts)
        dt = time.time() - t0
        rc, err = oracle_lib.verify(proof, pi, opts)
        assert rc == 0, err
        out[name] = {"seed": seed, "log_n": LOG_N, "flags": flags, "width": w,
                     "options": {f: getattr(opts, f) for f, _ in opts._fields_},
                     "len": len(proof), "sha256": hashlib.sha256(proof).hexdigest()}
        print(f"{name}: {len(proof)} bytes sha256 {out[name]['sha256'][:16]} ({dt:.0f}s)", flush=True)
        json.dump(out, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
