#!/usr/bin/env python3
"""bench.py — segment-proofs/s of the MI355X zk-lisp segment prover.

Workload (BASELINE.json configs[1] shape): one synthetic VM segment of 65,536 rows x 204
columns ({vm, rom} layout), blowup 16, q 64, grind 16, partitions (4, 16).  One step = one
full segment proof (trace LDE, constraint evaluation, composition, DEEP, FRI, grinding,
queries, Proof::to_bytes) with the trace already resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 is launched by torch.distributed.run, one rank per GPU; each rank proves its own
segments (weak scaling, no data-path collective).  The barrier and the
max-over-ranks timing (zkl_hip/dist.py) use torch.distributed's gloo backend: the
prover's HIP runtime (/opt/rocm 7.2) owns the device, and loading torch's bundled ROCm
runtime into the same process would create a second HIP runtime.
Device synchronisation is zkl_hip_synchronize (hipDeviceSynchronize) on both sides.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))

METRIC = "segment-proofs/sec at 65536 rows, blowup=16; proof bytes bit-exact vs CPU ref"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue peak: one wave64 VALU instruction per quad-cycle per SIMD (SQ_ACTIVE_INST_VALU
# counts one quad-cycle per instruction for this kernel's 64-bit integer mix), 256 CUs x 4
# SIMDs x 2.4 GHz / 4
VALU_ISSUE_PEAK_G = 256 * 4 * 2.4 / 4   # G wave-instructions/s
# VALU wave-instructions per Poseidon permutation of the trace row hash, from
# SQ_INSTS_VALU / permutations: matrix-core kernel hash_rows_pm_kernel<0> 1025
# (profiles/r01/pmc_sq_pm.json; the MDS runs on v_mfma_i32_32x32x32_i8), lane-group kernel
# hash_rows_kernel<0> 2617 (profiles/r01/pmc_sq_stagebench.json, ZKL_HASH_ENGINE=lane)
VALU_INSTR_PER_PERM = {"mfma": 1025, "lane": 2617}
ROW_KERNEL = {"mfma": "hash_rows_pm_kernel<0>", "lane": "hash_rows_kernel<0>"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def perm_model(n, W=204, C=7, blowup=16, parts=None, grind=16, n_tc=193, queries=64):
    """Algorithmic Poseidon permutation count of one segment proof (DESIGN.md §Work model)."""
    N = n * blowup
    if parts is None:
        parts = 16 if n >= 1 << 20 else 8 if n >= 1 << 18 else 4 if n >= 1 << 16 else 2 if n >= 1 << 14 else 1
    ceil = lambda a, b: -(-a // b)
    if parts == 1:
        row = ceil(ceil(W, 2) + 1, 10)
        crow = ceil(ceil(C, 2) + 1, 10)
    else:
        ps = max(ceil(W, parts), 16)
        np_ = ceil(W, ps)
        row = np_ * ceil(ceil(ps, 2) + 1, 10) + ceil(np_ + 1, 10)
        cps = max(ceil(C, parts), 16)
        crow = ceil(ceil(C, 2) + 1, 10) + (1 if cps != C else 0)
    n_assert = 141 * (n // 32) + 8
    fri = 0
    d = N
    while d > 2 * blowup:
        fri += d // 2 + (d // 2 - 1)
        d //= 2
    total = N * row + (N - 1) + N * crow + (N - 1) + fri + 2 ** grind + n_tc + n_assert + W + C + queries
    return {"trace_rows": N * row, "total": total, "row_perms": row}


MULMODS_PER_PERM = 27 * (144 + 24)  # f128 multiplications of one permutation (12 cubes x 2 + 144 MDS)


def cpu_baseline(log_n_sample, log_n_target, threads):
    """Oracle (CPU restatement of the reference algorithm) on a bounded sample: one full proof
    of the same synthetic segment family at 2^log_n_sample rows with `threads` OpenMP
    threads (row hashing, Merkle levels, LDE columns, constraint evaluation, DEEP, grinding
    in parallel), extrapolated to 2^log_n_target rows by the permutation-count work model."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc
    orc.lib()
    orc.set_threads(threads)
    n = 1 << log_n_sample
    t, pi, w = orc.synth_segment(0x5EED0001, log_n_sample)
    opts = orc.default_options(w, n)
    t0 = time.perf_counter()
    orc.prove(t, w, n, pi, opts)
    dt = time.perf_counter() - t0
    orc.set_threads(1)
    ms, mt = perm_model(n), perm_model(1 << log_n_target)
    per_target = dt * mt["total"] / ms["total"]
    return {
        "value": round(1.0 / per_target, 6),
        "unit": "segment-proofs/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"oracle proof of a 2^{log_n_sample}-row synthetic segment (same options) took {dt:.1f}s "
                   f"with {threads} threads; scaled x{mt['total'] / ms['total']:.2f} by the Poseidon-permutation "
                   f"work model to a 2^{log_n_target}-row segment"),
        "sample_seconds": round(dt, 2),
    }


def c5_single(zkl_hip, device, log_n):
    """BASELINE configs[4] shape on one GPU: one synthetic 2^log_n-row segment (blowup 16,
    q 64, grind 16, partitions (16,16) at 2^20 rows), trace resident in HBM; on 8 GPUs each
    rank proves its own segment (replicas).  One warm-up proof, one timed.
    Returns (ms per proof, proof bytes)."""
    n = 1 << log_n
    ctx = zkl_hip.Context(device)
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0C05, log_n)
    d = ctx.alloc(w * n * 16)
    ctx.upload(d, t, w * n * 16)
    del t
    o = zkl_hip.proof_options(w, n)
    ctx.prove_segment_device(d, w, n, pi, o)
    ctx.synchronize()
    t0 = time.perf_counter()
    proof = ctx.prove_segment_device(d, w, n, pi, o)
    ms = (time.perf_counter() - t0) * 1e3
    ctx.free(d)
    ctx.close()
    return ms, len(proof)


def c3_pipeline(zkl_hip, device, log_n, n_segments, inflight, reps=1):
    """BASELINE configs[2] shape: n_segments distinct 2^log_n-row segments proved on one GPU
    with `inflight` contexts (one HIP stream each) in host threads, so one segment's
    latency-bound tails (tree tops, FRI layers, transcript round trips) overlap another's
    throughput phases.  Traces are resident in HBM before timing.  Returns segments/s."""
    import threading
    n = 1 << log_n
    ctxs = [zkl_hip.Context(device) for _ in range(inflight)]
    segs = []
    for i in range(n_segments):
        t, pi, w = zkl_hip.synth_vm_segment(0x5EED0001 + i, log_n)
        c = ctxs[i % inflight]
        d = c.alloc(w * n * 16)
        c.upload(d, t, w * n * 16)
        segs.append((c, d, pi, w, zkl_hip.proof_options(w, n)))
    for k in range(inflight):  # warm each context (buffers, tables)
        c, d, pi, w, o = segs[k]
        c.prove_segment_device(d, w, n, pi, o)
    best = None
    for _ in range(reps):
        def run(k):
            for i in range(k, n_segments, inflight):
                c, d, pi, w, o = segs[i]
                c.prove_segment_device(d, w, n, pi, o)
        th = [threading.Thread(target=run, args=(k,)) for k in range(inflight)]
        for c in ctxs:
            c.synchronize()
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        for c in ctxs:
            c.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    for c, d, *_ in segs:
        c.free(d)
    for c in ctxs:
        c.close()
    return n_segments / best


def load_traffic(kernel):
    """HBM bytes per launch from the committed PMC summary (profiles/r01/pmc_traffic.json)."""
    p = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        return d.get(kernel)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--cpu-sample-log-n", type=int, default=14)
    ap.add_argument("--cpu-threads", type=int, default=0, help="oracle threads (0: min(16, host CPUs))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c3-segments", type=int, default=8, help="segments for the configs[2] pipeline line (0: skip)")
    ap.add_argument("--c3-inflight", type=str, default="1,2,4", help="contexts in flight to try for configs[2]")
    ap.add_argument("--c5-log-n", type=int, default=20, help="rows (log2) of the configs[4] single-segment line (0: skip)")
    args = ap.parse_args()

    # Only the result line goes to stdout: native libraries (gloo prints "[Gloo] Rank ..."
    # from C++) write to fd 1, so fd 1 is pointed at stderr and the JSON line is written
    # to a saved copy of the original stdout.
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    from zkl_hip import dist
    rank, world, local_rank = dist.init()  # gloo control plane only (zkl_hip/dist.py)

    import zkl_hip
    # ZKL_BENCH_DEVICE pins every rank to one device (rehearsing N > 1 on a 1-GPU box)
    device = int(os.environ.get("ZKL_BENCH_DEVICE", local_rank))
    ctx = zkl_hip.Context(device)
    log_n = args.log_n
    n = 1 << log_n
    trace, pi, W = zkl_hip.synth_vm_segment(0x5EED0001 + rank, log_n)
    opts = zkl_hip.proof_options(W, n)
    nbytes = W * n * 16
    d_trace = ctx.alloc(nbytes)
    ctx.upload(d_trace, trace, nbytes)
    log(f"[rank {rank}] trace {W}x{n} resident in HBM; warmup {args.warmup}")

    proof = None
    for _ in range(args.warmup):
        proof = ctx.prove_segment_device(d_trace, W, n, pi, opts)

    kacc = {}
    dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    step_ms = []
    for i in range(args.steps):
        proof = ctx.prove_segment_device(d_trace, W, n, pi, opts)
        step_ms.append(ctx.host_times()["call"])
        for k, (ms, cnt) in ctx.kernel_times().items():
            a = kacc.setdefault(k, [0.0, 0])
            a[0] += ms
            a[1] += cnt
    ctx.synchronize()
    dist.barrier()
    elapsed = dist.max_over_ranks(time.perf_counter() - t0)
    host = ctx.host_times()
    stages = {}
    # Inside the timed region only the dominant family (the trace row hash) is bracketed by
    # HIP events (each bracket costs ~10 us of queue time); one extra untimed proof with
    # every family bracketed gives the per-family breakdown.
    fam = {}
    if rank == 0:
        ctx.set_kernel_timing(2)
        ctx.prove_segment_device(d_trace, W, n, pi, opts)
        fam = ctx.kernel_times()
        stages = ctx.stage_times()
        ctx.set_kernel_timing(1)
    # Aggregation hand-off (untimed): every rank wraps its last proof as zl1
    # step `rank` of `world` (ZKLSTP1); rank 0 gathers, orders and chain-checks them and forms
    # the children root the aggregation proof commits to (agg/child.rs:853-895).
    t_h = time.perf_counter()
    info = zkl_hip.StepInfo()
    info.suite_id[:] = bytes(pi.program_id)
    info.lambda_bits, info.segment_index, info.segments_total = 128, rank, world
    info.state_in_hash[:] = rank.to_bytes(32, "little")  # synthetic chain: out(r) = in(r+1)
    info.state_out_hash[:] = (rank + 1).to_bytes(32, "little")
    steps = dist.collect_step_proofs([zkl_hip.step_proof_encode(pi, info, proof)])
    handoff = None
    if steps is not None:
        root = zkl_hip.children_root(bytes(pi.program_id), [d["digest"] for d in steps],
                                     [d["root_trace"] for d in steps])
        handoff = {"segments": len(steps), "step_bytes": sum(d["bytes"] for d in steps),
                   "ms": round((time.perf_counter() - t_h) * 1e3, 2), "children_root": root[:16].hex(),
                   "transport": "gloo (host bytes; the proofs already live in host memory)"}

    if rank == 0:
        value = world * args.steps / elapsed
        # dominant kernel family (from the breakdown proof) and its roofline (timed region)
        dom = max(fam.items(), key=lambda kv: kv[1][0])[0] if fam else "trace_hash_rows"
        ms_tot, launches = kacc["trace_hash_rows"]
        per_launch_ms = ms_tot / max(launches, 1)
        N = n * 16
        # fused partitioned row hash: the 2^20 x 204 LDE is read once, one digest per row written
        alg_bytes = W * N * 16 + N * 16
        achieved = alg_bytes / (per_launch_ms * 1e-3) / 1e9
        pm = perm_model(n)
        perms_per_launch = N * pm["row_perms"]  # fused: partitions + merge_many per row
        perms_per_s = perms_per_launch / (per_launch_ms * 1e-3)
        engine = "lane" if os.environ.get("ZKL_HASH_ENGINE") == "lane" else "mfma"
        kname = ROW_KERNEL[engine]
        valu_g = perms_per_s * VALU_INSTR_PER_PERM[engine] / 1e9
        traffic = load_traffic(kname)
        out = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "segment-proofs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f128 (u128 mod 2^128-45*2^40+1)",
            "data": "synthetic",
            "config": {
                "workload": f"synthetic VM segment {n} rows x {W} cols ({{vm,rom}} layout), blowup 16, q 64, "
                            f"grind 16, partitions ({opts.num_partitions},{opts.hash_rate}); trace resident in HBM",
                "rows": n, "width": W, "blowup": 16, "queries": 64, "grind": 16,
                "segments_per_gpu_per_step": 1, "parallelism": f"segments x{world} (one rank per GPU)",
                "proof_bytes": len(proof),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": f"{kname} (trace LDE row hashing, 4 partitions + merge_many)",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "alg_bytes_per_launch": alg_bytes,
                "avg_launch_ms": round(per_launch_ms, 3),
                "note": "VALU-issue bound (integer Poseidon); see roofline_valu",
            },
            "roofline_valu": {
                "bound": "valu-issue",
                "kernel": kname,
                "achieved": round(valu_g, 1),
                "peak": VALU_ISSUE_PEAK_G,
                "unit": "G VALU wave-instructions/s",
                "frac": round(valu_g / VALU_ISSUE_PEAK_G, 4),
                "perms_per_launch": perms_per_launch,
                "perms_per_s": round(perms_per_s),
                "f128_mulmods_per_s": round(perms_per_s * MULMODS_PER_PERM),
                "note": "VALU wave-instructions per permutation from SQ_INSTS_VALU (profiles/r01/pmc_sq_pm.json); "
                        "the 12x12 MDS runs on the matrix cores (MFMA busy ~21% of cycles)",
            },
            "dominant_kernel_family": dom,
            "kernel_ms_per_family_untimed_step": {k: round(v[0], 3) for k, v in fam.items()},
            "stage_ms_untimed_step": {k: round(v, 3) for k, v in stages.items()},
            "host_ms_last_step": {k: round(v, 3) for k, v in host.items()},
            "call_ms_each_step": [round(v, 2) for v in step_ms],
            "step_handoff": handoff,
        }
        if world == 1 and args.c3_segments > 0:
            c3 = {}
            for k in [int(x) for x in args.c3_inflight.split(",") if x]:
                c3[str(k)] = round(c3_pipeline(zkl_hip, device, log_n, args.c3_segments, k), 4)
            kbest = max(c3, key=lambda k: c3[k])
            out["c3_in_gpu_pipeline"] = {
                "config": f"BASELINE configs[2] shape: {args.c3_segments} distinct synthetic 2^{log_n}-row segments on 1 GPU",
                "segment_proofs_per_s_by_inflight": c3, "best_inflight": int(kbest), "value": c3[kbest],
                "unit": "segment-proofs/s"}
        if world == 1 and args.c5_log_n > 0:
            try:
                ms5, pb5 = c5_single(zkl_hip, device, args.c5_log_n)
                out["c5_single_segment"] = {
                    "config": f"BASELINE configs[4] shape on one GPU: one synthetic 2^{args.c5_log_n}-row segment, "
                              "blowup 16, q 64, grind 16 (each of the 8 GPUs proves its own)",
                    "ms_per_proof": round(ms5, 1), "proof_bytes": pb5,
                    "rows_per_s": round((1 << args.c5_log_n) / ms5 * 1e3)}
            except Exception as e:  # reported, never fatal for the headline number
                out["c5_single_segment"] = {"error": str(e)}
        if world == 1 and not args.no_cpu_baseline:
            try:
                th = args.cpu_threads or min(16, os.cpu_count() or 1)
                out["cpu_baseline"] = cpu_baseline(args.cpu_sample_log_n, log_n, th)
            except Exception as e:  # reported, never fatal for the GPU number
                out["cpu_baseline"] = {"value": None, "error": str(e)}
        print(json.dumps(out), file=result_out, flush=True)
    ctx.free(d_trace)
    ctx.close()
    dist.shutdown()


if __name__ == "__main__":
    main()
