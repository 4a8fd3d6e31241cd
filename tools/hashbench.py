#!/usr/bin/env python3
"""Throughput of the Poseidon stage kernels through the C ABI (zkl_hip_hash_rows /
zkl_hip_merkle_tree), for comparing kernel variants on the GPU box.

  ZKL_HIP_LIB=path/to/libzkl_hip.so python tools/hashbench.py [--log-rows 20] [--reps 3]

Prints one JSON line: ms per call and Poseidon permutations/s for
  rows  : hash_rows over a 204-column x 2^log_rows matrix, 4 partitions (trace commitment)
  ntt   : zkl_hip_ntt DIT over the same 204 columns (all log_rows stages)
  comp  : hash_rows over 7 columns, 4 partitions (composition commitment)
  tree  : full Merkle tree over 2^log_rows leaves
Inputs are arbitrary field elements (< p); only timing is of interest here.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-rows", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="comma list of: rows,comp,tree,perm,ntt (default all)")
    args = ap.parse_args()
    import numpy as np
    import zkl_hip

    n = 1 << args.log_rows
    ctx = zkl_hip.Context(0)
    rng = np.random.default_rng(1)
    W = 204
    host = rng.integers(0, 2**63, size=(W * n * 2,), dtype=np.uint64)
    d_mat = ctx.alloc(host.nbytes)
    ctx.upload(d_mat, host.ctypes.data, host.nbytes)
    d_out = ctx.alloc(n * 16)
    d_nodes = ctx.alloc(2 * n * 16)

    def timeit(fn):
        fn()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        ctx.synchronize()
        return (time.perf_counter() - t0) / args.reps * 1e3

    out = {"lib": os.environ.get("ZKL_HIP_LIB", "default"), "rows": n}
    only = set(args.only.split(",")) if args.only else {"rows", "comp", "tree", "perm", "ntt"}
    if "rows" in only:
        ms = timeit(lambda: ctx.hash_rows(d_mat, W, n, 4, 16, d_out))
        perms = n * (4 * 3 + 1)
        out["rows_ms"] = round(ms, 3)
        out["rows_Mperm_s"] = round(perms / ms / 1e3, 1)
    if "comp" in only:
        ms = timeit(lambda: ctx.hash_rows(d_mat, 7, n, 4, 16, d_out))
        out["comp_ms"] = round(ms, 3)
        out["comp_Mperm_s"] = round(2 * n / ms / 1e3, 1)
    if "tree" in only:
        ms = timeit(lambda: ctx.merkle_tree(d_out, n, d_nodes))
        out["tree_ms"] = round(ms, 3)
        out["tree_Mperm_s"] = round((n - 1) / ms / 1e3, 1)
    # raw permutations (2^log_rows states) in both forms
    if "perm" in only:
        d_st = ctx.alloc(n * 12 * 16)
        ctx.upload(d_st, host.ctypes.data, n * 12 * 16)
        for eng, name in ((1, "perm_mfma"), (0, "perm_lane")):
            ms = timeit(lambda: ctx.poseidon_permute(d_st, n, eng))
            out[name + "_ms"] = round(ms, 3)
            out[name + "_Mperm_s"] = round(n / ms / 1e3, 1)
        ctx.free(d_st)
    if "ntt" in only:  # W columns of 2^log_rows, DIT (bit-reversed -> natural), all stages
        ms = timeit(lambda: ctx.ntt(d_mat, W, n, dif=False))
        out["ntt_dit_ms"] = round(ms, 3)
        out["ntt_Gbfly_s"] = round(W * (n // 2) * args.log_rows / ms / 1e6, 1)
    print(json.dumps(out), flush=True)
    for p in (d_mat, d_out, d_nodes):
        ctx.free(p)
    ctx.close()


if __name__ == "__main__":
    main()
