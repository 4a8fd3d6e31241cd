#!/usr/bin/env python3
"""bench.py — segment-proofs/s of the MI355X zk-lisp segment prover.

Workload (BASELINE.json configs[1] shape): one synthetic VM segment of 65,536 rows x 204
columns ({vm, rom} layout), blowup 16, q 64, grind 16, partitions (4, 16).  One step = one
full segment proof per rank (trace LDE, constraint evaluation, composition, DEEP, FRI,
grinding, queries, Proof::to_bytes) with the trace already resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--segments S] [--dry-run]

Ranks.  N > 1 runs one process per GPU.  Under torch.distributed.run (RANK / WORLD_SIZE set)
this process is one rank and WORLD_SIZE must equal --gpus.  Started directly with --gpus N > 1
and no WORLD_SIZE, this process is only a launcher: before touching any GPU it starts N child
processes of itself with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT
set, relays rank 0's JSON line and exits non-zero if any rank fails.  Rank r proves segment
seed 0x5EED0001 + r on device LOCAL_RANK (ZKL_BENCH_DEVICE pins every rank to one device to
rehearse N ranks on fewer GPUs; the JSON line then says so).  Weak scaling, no data-path
collective.  The step-proof hand-off to rank 0 runs over RCCL (zkl_comm_*,
ncclSend/ncclRecv over xGMI); with one GPU per rank RCCL is required, and a failure to start it
or to gather ends the run non-zero.  gloo carries the barrier, the max-over-ranks timing and the
RCCL unique id, and carries the step bytes only in a same-device rehearsal (ZKL_BENCH_DEVICE) or
with ZKL_COMM=gloo, which the line's handoff.transport states (zkl_hip/dist.py).

Parity.  Every rank hashes its last proof and compares it with the committed CPU-oracle
golden of its segment (tests/golden/proof_2p16.json, make_proof_goldens.py); at N = 1 the
cpu_baseline leg also proves the same segment on the oracle and compares the bytes.

Other lines: configs[2] (8 distinct segments on one GPU, 1/2/4 contexts in flight), configs[3]
shape (--segments S distinct segments sharded over the ranks, each rank pipelining its share,
then the step-proof gather and children root on rank 0; default S = 8 x N when N > 1),
configs[4] (one 2^20-row segment per rank: replicas, max-over-ranks time) and the real program
examples/rollup-bench.zlisp at --max-segment-rows 65536 (one 65,536-row x 212-column segment
built from the compiler's op list, tests/golden/programs.json; N = 1).  Device synchronisation is zkl_hip_synchronize
(hipDeviceSynchronize) on both sides of every timed region.
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))

T_START = time.time()
METRIC = "segment-proofs/sec at 65536 rows, blowup=16; proof bytes bit-exact vs CPU ref"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SEED0 = 0x5EED0001             # segment seed of rank / segment 0
GOLDEN = os.path.join(ROOT, "tests", "golden", "proof_2p16.json")
CHAIN = os.path.join(ROOT, "tests", "golden", "chain_2p16.json")  # the multi-segment program (make_chain_goldens.py)
PROGRAMS = os.path.join(ROOT, "tests", "golden", "programs.json")  # real .zlisp programs (make_programs.py)
FIB = os.path.join(ROOT, "tests", "golden", "fib_2pow16.json")  # examples/fib-2pow16.zlisp (make_fib_2pow16.py)
VALU_MIX = os.path.join(ROOT, "profiles", "r04", "valu_mix.json")
VALU_FLOOR = os.path.join(ROOT, "profiles", "r03", "valu_floor.json")
ROW_KERNEL = {"mfma": "hash_rows_pm_kernel<0>", "lane": "hash_rows_kernel<0>"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def perm_model(n, W=204, C=7, blowup=16, parts=None, grind=16, n_tc=193, queries=64):
    """Algorithmic Poseidon permutation count of one segment proof (DESIGN.md §5 work model)."""
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


def golden_sha(seed, log_n):
    """sha256 of the oracle proof of segment `seed` at the headline options, if committed."""
    if log_n != 16 or not os.path.exists(GOLDEN):
        return None
    for v in json.load(open(GOLDEN)).values():
        if v["seed"] == seed and v["flags"] == 0 and v["log_n"] == log_n:
            return v["sha256"]
    return None


def parity_of(proof, seed, log_n):
    want = golden_sha(seed, log_n)
    got = hashlib.sha256(proof).hexdigest()
    return {"seed": hex(seed), "sha256": got, "golden": "match" if want == got else ("none" if want is None else "MISMATCH")}


def chain_table():
    try:
        return json.load(open(CHAIN))
    except (OSError, ValueError):
        return None


def chain_segment(zkl_hip, i, log_n):
    """Segment i of the synthetic multi-segment program (tests/golden/chain_2p16.json): program
    seed P, ops seed P + i, ROM lane 0 entering where segment i - 1 ended.  The committed table
    gives every segment's entry value, so a rank builds only its own segments."""
    tab = chain_table()
    if tab is None or log_n != tab["log_n"] or i >= len(tab["rom0_in"]):
        raise RuntimeError(f"no chain table entry for segment {i} at 2^{log_n} rows (run make_chain_goldens.py)")
    return zkl_hip.synth_vm_segment_chain(tab["program_seed"], tab["program_seed"] + i, log_n, int(tab["rom0_in"][i], 16))


def chain_parity(i, proof):
    tab = chain_table() or {}
    want = next((s["sha256"] for s in tab.get("segments", []) if s["index"] == i), None)
    got = hashlib.sha256(proof).hexdigest()
    return "match" if want == got else ("none" if want is None else "MISMATCH")


def chain_step(zkl_hip, i, total, pi, proof):
    """zl1 step proof of chain segment i of `total` (VM state hashes state_in = i, state_out = i + 1)."""
    info = zkl_hip.step_info_for(pi, i, total, i.to_bytes(32, "little"), (i + 1).to_bytes(32, "little"))
    return zkl_hip.step_proof_encode(pi, info, proof)


def aggregate(zkl_hip, steps):
    """The aggregation proof over the gathered step proofs (zkl_agg_prove: build_public +
    RecursionBackend::prove + ZKLRC1 encode, lib.rs:295-551), host-side on rank 0."""
    t0 = time.perf_counter()
    art, dg = zkl_hip.agg_prove(steps)
    ms = (time.perf_counter() - t0) * 1e3
    out = {"children": len(steps), "ms": round(ms, 1), "artifact_bytes": len(art), "recursion_digest": dg.hex(),
           "field_extension": "quadratic (min_security_bits 128)"}
    tab = chain_table() or {}
    for key in ("aggregation", "aggregation_64"):  # the 8-child (configs[2]) and 64-child (configs[3]) artifacts
        g = tab.get(key)
        if g and g["children"] == len(steps):
            out["golden"] = "match" if g["sha256"] == hashlib.sha256(art).hexdigest() else "MISMATCH"
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_affinity():
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_threads(requested):
    """Threads of the CPU baseline: the CPUs this process can actually use -- the cores it may
    run on (sched_getaffinity) capped by the cgroup's CPU quota (cpu.max).  On the GPU box the
    affinity mask lists every core of the host (256 on the EPYC 9575F node) while the quota
    grants 16 CPUs' worth of time; one proof on 256 threads there measured 96.9 s against
    ~37 s on 16 (profiles/r03/cpu_baseline_threads.json), so the quota is the core count the
    host gives this run.  --cpu-threads overrides."""
    if requested:
        return requested
    n = cpu_affinity()
    q = cgroup_cpu_quota()
    return max(1, min(n, int(q))) if q else n


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants (cpu.max quota / period), or None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(log_n, threads, gpu_proof, log_n_target):
    """Oracle (oracle/, the CPU restatement of the reference algorithm) proving the bench's own
    segment (seed SEED0, same options) with `threads` OpenMP threads inside the one proof (row
    hashing, Merkle levels, LDE columns, constraint evaluation, DEEP, grinding in parallel).
    At log_n == log_n_target this is the measured CPU rate of the headline workload, and its
    proof bytes are compared with the GPU proof of the same segment."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc
    orc.lib()
    orc.set_threads(threads)
    n = 1 << log_n
    t, pi, w = orc.synth_segment(SEED0, log_n)
    opts = orc.default_options(w, n)
    t0 = time.perf_counter()
    proof = orc.prove(t, w, n, pi, opts)
    dt = time.perf_counter() - t0
    stages = dict(zip(("trace_lde", "trace_commit", "evaluator", "constraint_commitment", "deep", "fri",
                       "grind", "queries"), (round(x / 1e3, 3) for x in orc.last_times())))
    orc.set_threads(1)
    out = {"unit": "segment-proofs/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
           "cores_in_affinity_mask": cpu_affinity(), "cgroup_cpu_quota": cgroup_cpu_quota(),
           "mode": "one proof using every thread (row hashing, Merkle levels, LDE columns, constraint "
                   "evaluation, DEEP and grinding split over the threads)",
           "sample_seconds": round(dt, 2), "stage_seconds": stages}
    if log_n == log_n_target:
        out["value"] = round(1.0 / dt, 6)
        out["sample"] = (f"one full oracle proof of the headline segment (2^{log_n} rows x {w} cols, blowup 16, q 64, "
                         f"grind 16, partitions ({opts.num_partitions},{opts.hash_rate})) using {threads} threads "
                         f"inside the proof; measured, not extrapolated")
        out["proof_equals_gpu_proof"] = (proof == gpu_proof) if gpu_proof is not None else None
    else:
        ms, mt = perm_model(n), perm_model(1 << log_n_target)
        out["value"] = round(1.0 / (dt * mt["total"] / ms["total"]), 6)
        out["sample"] = (f"EXTRAPOLATED: oracle proof of a 2^{log_n}-row segment with {threads} threads took "
                         f"{dt:.1f}s, scaled x{mt['total'] / ms['total']:.2f} by the permutation work model")
    return out


def valu_roofline(perms_per_s):
    """Achieved permutations/s of the row hash against the ceiling its own instruction mix
    implies at the measured per-class VALU rates (tools/valu_mix.py -> profiles/r04/valu_mix.json)."""
    try:
        mix = json.load(open(VALU_MIX))
    except (OSError, ValueError):
        return None
    peak = mix["peak_perms_per_s"]
    try:
        floor = json.load(open(VALU_FLOOR))
    except (OSError, ValueError):
        floor = None
    extra = {}
    if floor:
        extra = {"algorithm_floor_perms_per_s_M": round(floor["floor_perms_per_s"] / 1e6, 1),
                 "frac_of_algorithm_floor": round(perms_per_s / floor["floor_perms_per_s"], 4),
                 "algorithm_valu_per_element_round": floor["valu_per_element_round"],
                 "kernel_valu_per_element_round": floor["kernel_valu_per_element_round"]}
    return {"bound": "valu-issue (instruction-mix ceiling)", "kernel": mix["kernel"], **extra,
            "achieved": round(perms_per_s / 1e6, 1), "peak": round(peak / 1e6, 1), "unit": "M permutations/s",
            "frac": round(perms_per_s / peak, 4),
            "valu_per_perm_round_loop": mix["valu_per_perm_round_loop"],
            "f128_mulmods_per_s": round(perms_per_s * MULMODS_PER_PERM),
            "note": "peak = 32/27 wave-rounds per sum_c(count_c / rate_c) over the round loop's VALU classes, "
                    "rates measured by tools/madbench.hip (profiles/r01/madbench.txt); the 12x12 MDS runs on "
                    "v_mfma_i32_32x32x32_i8 and is not VALU work"}


def load_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary of the newest round."""
    for r in ("r06", "r05", "r04", "r03", "r02", "r01"):
        p = os.path.join(ROOT, "profiles", r, "pmc_traffic.json")
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if kernel in d:
            return d[kernel]
    return None


# ------------------------------------------------------------------------ launcher
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """--gpus n without a torch.distributed.run environment: start n ranks of this script as
    child processes (fresh interpreters; this process never initialises HIP), relay rank 0's
    stdout, return non-zero if any rank fails."""
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))
    out0 = procs[0].stdout.read()
    rcs = [p.wait() for p in procs]
    if any(rcs):
        log(f"bench: rank exit codes {rcs}")
        return next(rc for rc in rcs if rc) if all(rc >= 0 for rc in rcs) else 1
    sys.stdout.buffer.write(out0)
    sys.stdout.flush()
    return 0


def lines_for_rank(args, world):
    """The bench lines every rank takes part in (the --dry-run report; main() runs the same)."""
    lines = ["headline", "step_handoff"]
    n_seg = args.segments if args.segments >= 0 else (8 * world if world > 1 else 0)
    if n_seg > 0:
        lines.append("c4_sharded")
    if args.c5_log_n > 0:
        lines.append("c5_single_segment")
    lines += [f"program:{p}" for p in program_specs(args)]
    if world == 1:
        lines += [x for x, on in (("host_trace", args.host_steps > 0), ("c3_in_gpu_pipeline", args.c3_segments > 0),
                                  ("real_program", args.program_steps > 0),
                                  ("cpu_baseline", not args.no_cpu_baseline)) if on]
    return lines


def program_specs(args):
    if args.programs in ("", "none"):
        return []
    return [p for p in args.programs.split(",") if p]


# ------------------------------------------------------------------------ workloads
def c5_single(zkl_hip, device, log_n, barrier=lambda: None, seed=0x5EED0C05):
    """BASELINE configs[4] shape on one GPU: one synthetic 2^log_n-row segment (blowup 16,
    q 64, grind 16, partitions (16,16) at 2^20 rows), trace resident in HBM; on N GPUs every
    rank proves its own segment (replicas) between barriers.  One warm-up proof,
    one timed.  Every rank passes both barriers even if its own setup or proof fails, so a
    failing rank cannot leave the others waiting.  Returns (ms per proof, proof bytes, error)."""
    n = 1 << log_n
    ctx = d = None
    err = ms = nbytes = None
    try:
        ctx = zkl_hip.Context(device)
        t, pi, w = zkl_hip.synth_vm_segment(seed, log_n)
        d = ctx.alloc(w * n * 16)
        ctx.upload(d, t, w * n * 16)
        del t
        o = zkl_hip.proof_options(w, n)
        ctx.prove_segment_device(d, w, n, pi, o)
        ctx.synchronize()
    except Exception as e:  # noqa: BLE001  (reported in the line)
        err = str(e)
    barrier()
    if err is None:
        try:
            t0 = time.perf_counter()
            proof = ctx.prove_segment_device(d, w, n, pi, o)
            ctx.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            nbytes = len(proof)
        except Exception as e:  # noqa: BLE001
            err = str(e)
    barrier()
    if ctx is not None:
        if d is not None:
            ctx.free(d)
        ctx.close()
    return ms, nbytes, err


def real_program(zkl_hip, device, steps, name="rollup-bench", max_rows=1 << 16):
    """The reference's own example program at the metric's shape: `zk-lisp prove
    examples/<name>.zlisp --max-segment-rows 65536` with the CLI's arguments.  The op list is
    the compiler's (tests/golden/programs.json, lowered by oracle/lower_ref.py from the source
    and committed as data); the product builds the trace (zkl_build_trace), plans and slices the
    segment (zkl_plan_segments / zkl_slice_segment: one 65,536-row segment, {vm, ram, sponge,
    rom} layout, 212 columns), uploads it and proves it `steps` times resident in HBM.  The
    proof bytes are compared with the oracle's golden."""
    tab = json.load(open(PROGRAMS))[name]
    plan_g = tab["plans"][str(max_rows)]
    ops = [zkl_hip.op(k, **f) for k, f in tab["ops"]]
    main_args = [(tg, bytes.fromhex(b)) for tg, b in tab["cli"]["main_args"]]
    t, pi, w, n = zkl_hip.build_trace(ops, bytes.fromhex(tab["program_id"]), secret_args=tab["cli"]["secret_u64"],
                                      main_args=main_args)
    plan = zkl_hip.plan_segments(len(ops), max_rows)
    if [list(p) for p in plan] != [s["rows"] for s in plan_g["segments"]] or len(plan) != 1:
        raise RuntimeError(f"{name}: plan {plan} differs from the golden plan")
    a, b = plan[0]
    st, spi, sw, _, _ = zkl_hip.slice_segment(t, w, n, ops, pi, a, b)
    del t
    m = b - a
    cli = tab["cli"]
    o = zkl_hip.proof_options(sw, m, queries=cli["queries"], blowup=cli["blowup"], grind=cli["grind"])
    ctx = zkl_hip.Context(device)
    d = ctx.alloc(sw * m * 16)
    ctx.upload(d, st, sw * m * 16)
    del st
    try:
        ctx.prove_segment_device(d, sw, m, spi, o)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            proof = ctx.prove_segment_device(d, sw, m, spi, o)
        ctx.synchronize()
        dt = time.perf_counter() - t0
        ctx.set_kernel_timing(2)  # per-family breakdown from one extra, untimed proof
        ctx.prove_segment_device(d, sw, m, spi, o)
        fam = {k: round(v[0], 3) for k, v in ctx.kernel_times().items()}
    finally:
        ctx.free(d)
        ctx.close()
    want = plan_g["segments"][0]["proof_sha256"]
    got = hashlib.sha256(proof).hexdigest()
    return {"config": f"examples/{name}.zlisp (--arg u64:10 --arg bytes32:0x01), --max-segment-rows {max_rows}: "
                      f"one {m}-row x {sw}-column segment (feature mask {spi.segment_feature_mask:#x}: vm, ram, "
                      f"sponge, rom), blowup {cli['blowup']}, q {cli['queries']}, grind {cli['grind']}, "
                      f"partitions ({o.num_partitions},{o.hash_rate}); op list from the compiler restatement",
            "value": round(steps / dt, 4), "unit": "segment-proofs/s", "ms_per_proof": round(dt / steps * 1e3, 3),
            "steps": steps, "rows": m, "width": sw, "proof_bytes": len(proof),
            "parity": "match" if got == want else "MISMATCH", "golden": "tests/golden/programs.json (CPU oracle)",
            "kernel_ms_per_family_untimed_step": fam}


def load_program(zkl_hip, name):
    """(ops, program_id, secret u64 args, main args, max_rows -> {segment index: golden}) of a real
    example: rollup-bench / fib-2pow16-log-n from tests/golden/programs.json, fib-2pow16 from
    tests/golden/fib_2pow16.json and its gzip'd op list (the compiler's output, committed as data)."""
    if name == "fib-2pow16":
        import gzip
        g = json.load(open(FIB))
        raw = gzip.open(os.path.join(os.path.dirname(FIB), g["ops_file"])).read()
        if hashlib.sha256(raw).hexdigest() != g["ops_json_sha256"]:
            raise RuntimeError("fib-2pow16 op list fixture does not match its sha256")
        ops = [zkl_hip.op(k, **f) for k, f in json.loads(raw)]
        gold = {g["max_segment_rows"]: {int(k): v for k, v in g["segments"].items()}}
        return ops, bytes.fromhex(g["program_id"]), [], [], gold
    tab = json.load(open(PROGRAMS))[name]
    ops = [zkl_hip.op(k, **f) for k, f in tab["ops"]]
    main_args = [(tg, bytes.fromhex(b)) for tg, b in tab["cli"]["main_args"]]
    gold = {int(mr): dict(enumerate(p["segments"])) for mr, p in tab["plans"].items()}
    aggs = {int(mr): p.get("aggregation", {}) for mr, p in tab["plans"].items()}
    return ops, bytes.fromhex(tab["program_id"]), tab["cli"]["secret_u64"], main_args, gold, aggs


def program_sharded(zkl_hip, dist, device, rank, world, name, max_rows, inflight, builders, resident=False):
    """`zk-lisp prove examples/<name>.zlisp --max-segment-rows <max_rows>` sharded over the ranks
    (segment i on rank i mod N, prove.rs:1018-1050's pool per rank): each rank runs the program
    once (zkl_program_new), builds only its own segments (zkl_build_segment_trace, no full trace)
    on `builders` host threads straight into pinned trace buffers and proves them through the
    host-trace entry point with `inflight` contexts (zkl_hip.program.prove_program) -- timed end
    to end between barriers, value = segments / max-over-ranks seconds.  Then the zl1 steps go to
    rank 0 over RCCL, which checks the VM-state chain and proves the aggregation.  At N = 1 with
    `resident`, the same segments are also proved from HBM-resident traces (the headline's
    definition: trace already on the device).  A failing rank still passes every barrier and
    collective (the error flag is reduced over the ranks first), so no rank is left waiting."""
    from zkl_hip.program import prove_program, steps_of
    err, ctxs, P, plan, dt, par, res_line, enc = None, [], None, [], 0.0, [], None, []
    build_ms = prove_ms = [0.0]
    run_s = 0.0
    aggs = {}
    try:
        loaded = load_program(zkl_hip, name)
        ops, pid, secret, main_args, gold = loaded[:5]
        aggs = loaded[5] if len(loaded) > 5 else {}
        t_run = time.perf_counter()
        P = zkl_hip.Program(ops, pid, secret_args=secret, main_args=main_args)
        run_s = time.perf_counter() - t_run
        plan = zkl_hip.plan_segments(len(ops), max_rows)
        mine = dist.segments_for_rank(len(plan), rank, world)
        ctxs = [zkl_hip.Context(device) for _ in range(inflight)]
        prove_program(P, plan, segments=mine[:inflight], contexts=ctxs, builders=builders)  # warm contexts
    except Exception as e:  # noqa: BLE001
        err = f"setup: {e}"
    dist.barrier()
    if err is None:
        try:
            t0 = time.perf_counter()
            recs = prove_program(P, plan, segments=mine, contexts=ctxs, builders=builders)
            dt = time.perf_counter() - t0
            g = gold.get(max_rows, {})
            par = [("match" if hashlib.sha256(r.proof).hexdigest() == g[i]["proof_sha256"] else "MISMATCH")
                   for i, r in recs.items() if i in g]
            build_ms = sorted(r.build_ms for r in recs.values())
            prove_ms = sorted(r.prove_ms for r in recs.values())
            enc = steps_of(list(recs.values()), len(plan), main_args=main_args)
        except Exception as e:  # noqa: BLE001
            err = f"prove: {e}"
    dist.barrier()
    el = dist.max_over_ranks(dt)
    failed = dist.max_over_ranks(1.0 if err else 0.0) > 0
    par_all = dist.gather_to_root(par)
    errs = [e for e in (dist.gather_to_root(err) or []) if e]
    if not failed and resident and world == 1:
        try:
            res_line = program_resident(zkl_hip, ctxs, P, plan, mine, builders)
        except Exception as e:  # noqa: BLE001
            res_line = {"error": str(e)}
    for c in ctxs:
        c.close()
    if failed:
        return {"error": "; ".join(f"rank {i}: {e}" for i, e in enumerate(errs))} if rank == 0 else None
    comm, cerr = dist.init_rccl(device)
    t_h = time.perf_counter()
    steps = dist.collect_step_proofs(enc, comm)
    if rank != 0:
        return None
    flat = [x for r in par_all for x in r]
    widths = sorted({P.segment_width(a, b) for a, b in plan})
    out = {"config": f"examples/{name}.zlisp --max-segment-rows {max_rows}: {len(plan)} segments of "
                     f"{plan[0][1] - plan[0][0]} rows (widths {widths}), blowup 16, q 64, grind 16, sharded over "
                     f"{world} rank(s), {inflight} contexts in flight per rank; traces built per segment "
                     "(zkl_build_segment_trace) into pinned buffers and proved through zkl_hip_prove_segment",
           "value": round(len(plan) / el, 4), "unit": "segment-proofs/s", "seconds": round(el, 3),
           "segments": len(plan), "program_run_s": round(run_s, 2),
           "build_ms_per_segment_median": round(build_ms[len(build_ms) // 2], 1),
           "prove_call_ms_median": round(prove_ms[len(prove_ms) // 2], 1),
           "golden_matches": flat.count("match"), "golden_mismatches": flat.count("MISMATCH"),
           "handoff": {"ms": round((time.perf_counter() - t_h) * 1e3, 1),
                       "transport": "rccl" if comm is not None else f"gloo ({cerr})",
                       "step_bytes": sum(d["bytes"] for d in steps)}}
    if res_line is not None:
        out["resident"] = res_line
    out["aggregation"] = program_aggregation(zkl_hip, [d["raw"] for d in steps], aggs.get(max_rows, {}))
    return out


def program_aggregation(zkl_hip, raw, gold):
    """The aggregation over a program's gathered steps (valid trace mode, then verified), checked
    against the oracle's artifacts where the goldens hold them.  A batch the valid mode must refuse
    (tests/golden/programs.json "rejected": rollup-bench at 1024 rows cuts its sorted RAM table,
    DESIGN.md §10) is refused here too, and the reference trace mode's artifact is compared."""
    a = {"children": len(raw)}
    want = gold.get("valid", {})
    try:
        t1 = time.perf_counter()
        art, _ = zkl_hip.agg_prove(raw)
        a.update(ms=round((time.perf_counter() - t1) * 1e3, 1), artifact_bytes=len(art))
        zkl_hip.agg_verify(art)
        a["verified"] = True
        if "sha256" in want:
            a["golden"] = "match" if hashlib.sha256(art).hexdigest() == want["sha256"] else "MISMATCH"
        elif "rejected" in want:
            a["golden"] = "MISMATCH"
            a["error"] = "the valid mode accepted a batch the oracle rejects"
    except Exception as e:  # noqa: BLE001
        if "rejected" not in want:
            return {"error": str(e)}
        a["valid_mode"] = f"rejected, as by the oracle: {e}"
    ref = gold.get("reference_trace")
    if ref and "sha256" in ref:
        t1 = time.perf_counter()
        art, _ = zkl_hip.agg_prove(raw, trace_mode=zkl_hip.AGG_TRACE_REFERENCE)
        a["reference_trace"] = {"ms": round((time.perf_counter() - t1) * 1e3, 1), "artifact_bytes": len(art),
                                "golden": "match" if hashlib.sha256(art).hexdigest() == ref["sha256"] else "MISMATCH"}
        if a["reference_trace"]["golden"] == "MISMATCH":
            a["golden"] = "MISMATCH"
    return a


def program_resident(zkl_hip, ctxs, P, plan, idx, builders):
    """The program's segments built on `builders` host threads, uploaded (all resident in HBM:
    256 x 214 MB = 55 GB for fib-2pow16) and proved from HBM by the contexts in flight: the
    headline's definition of a step (trace already on the device)."""
    import threading
    from concurrent.futures import ThreadPoolExecutor
    inflight = len(ctxs)
    segs = []
    try:
        win = 2 * max(1, builders)  # host traces alive at once
        with ThreadPoolExecutor(max_workers=max(1, builders)) as ex:
            futs = {k: ex.submit(P.segment, *plan[i]) for k, i in enumerate(idx[:win])}
            for k in range(len(idx)):
                t, pi, w, _, _ = futs.pop(k).result()
                if k + win < len(idx):
                    futs[k + win] = ex.submit(P.segment, *plan[idx[k + win]])
                m = len(t) // w
                c = ctxs[k % inflight]
                d = c.alloc(w * m * 16)
                c.upload(d, t, w * m * 16)
                segs.append((c, d, pi, w, m, zkl_hip.proof_options(w, m)))
                del t

        def work(k):
            for c, d, pi, w, m, o in segs[k::inflight]:
                c.prove_segment_device(d, w, m, pi, o)

        th = [threading.Thread(target=work, args=(k,)) for k in range(inflight)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        for c in ctxs:
            c.synchronize()
        dt = time.perf_counter() - t0
    finally:
        for c, d, *_ in segs:
            c.free(d)
    return {"value": round(len(segs) / dt, 4), "unit": "segment-proofs/s", "seconds": round(dt, 3),
            "note": "every segment's trace resident in HBM before the timed region; same contexts in flight"}


class Pipeline:
    """A set of distinct segments resident in HBM, proved by `inflight` contexts (one HIP
    stream each) in host threads, so one segment's latency-bound tails (tree tops, FRI
    layers, transcript round trips) overlap another's throughput phases (BASELINE configs[2];
    the reference's bounded segment pool, prove.rs:1018-1050)."""

    def __init__(self, zkl_hip, device, log_n, seg_ids, inflight):
        self.n = 1 << log_n
        self.ctxs = [zkl_hip.Context(device) for _ in range(inflight)]
        self.segs = []
        for k, i in enumerate(seg_ids):
            t, pi, w = chain_segment(zkl_hip, i, log_n)
            c = self.ctxs[k % inflight]
            d = c.alloc(w * self.n * 16)
            c.upload(d, t, w * self.n * 16)
            self.segs.append([i, c, d, pi, w, zkl_hip.proof_options(w, self.n), None])
        for k in range(min(inflight, len(self.segs))):  # warm each context (buffers, tables)
            _, c, d, pi, w, o, _ = self.segs[k]
            c.prove_segment_device(d, w, self.n, pi, o)

    def run(self):
        import threading
        inflight = len(self.ctxs)

        def work(k):
            for s in self.segs[k::inflight]:
                s[6] = s[1].prove_segment_device(s[2], s[4], self.n, s[3], s[5])

        th = [threading.Thread(target=work, args=(k,)) for k in range(inflight)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        for c in self.ctxs:
            c.synchronize()

    def proofs(self):
        return [(s[0], s[3], s[6]) for s in self.segs]

    def close(self):
        for s in self.segs:
            s[1].free(s[2])
        for c in self.ctxs:
            c.close()


def host_inflight(zkl_hip, device, trace, W, n, pi, opts, steps):
    """Two contexts proving concurrently (the reference's rayon pool calls prove_segment from
    several threads, prove.rs:1020-1048): the same K proofs per context once from the host trace
    (zkl_hip_prove_segment, each upload overlapping the other context's compute) and once from a
    copy resident in HBM (zkl_hip_prove_segment_device).  Returns both rates and their ratio."""
    import threading
    ctxs = [zkl_hip.Context(device) for _ in range(2)]
    nbytes = W * n * 16
    dev = []
    try:
        for c in ctxs:
            d = c.alloc(nbytes)
            c.upload(d, trace, nbytes)
            dev.append(d)
            c.prove_segment(trace, W, n, pi, opts)  # warm (buffers, tables, pinned ring)

        def rate(host):
            def work(k):
                for _ in range(steps):
                    if host:
                        ctxs[k].prove_segment(trace, W, n, pi, opts)
                    else:
                        ctxs[k].prove_segment_device(dev[k], W, n, pi, opts)
            th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
            t0 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            for c in ctxs:
                c.synchronize()
            return 2 * steps / (time.perf_counter() - t0)

        r_dev, r_host = rate(False), rate(True)
    finally:
        for c, d in zip(ctxs, dev):
            c.free(d)
        for c in ctxs:
            c.close()
    return {"host_trace": round(r_host, 4), "resident": round(r_dev, 4), "unit": "segment-proofs/s",
            "fraction_of_resident_rate": round(r_host / r_dev, 4)}


def host_fresh(zkl_hip, device, trace, W, n, pi, opts, steps):
    """The Rust binding's allocation pattern (prove.rs:1103-1142: a fresh TraceTable per segment,
    filled, proved, dropped): two contexts in flight, each proof from a newly malloc'd host trace
    (214 MB, filled with a copy of the trace, freed after its proof) -- against the same with the
    contexts' pinned trace buffers (zkl_hip_trace_buffer, two slots, filled in place, nothing
    allocated per proof), and a fresh allocation the caller advises onto transparent huge pages
    (madvise MADV_HUGEPAGE before the fill).  Per-proof call times: median and slowest / median
    (stalled proofs), and the median of each phase of a call: malloc, fill (the
    caller's first touch of fresh pages for fresh allocations), the library call
    (zkl_hip_prove_segment: staging copies, DMA, proof; its upload loop separately) and free."""
    import ctypes as C
    import threading
    libc = C.CDLL("libc.so.6", use_errno=True)
    libc.malloc.restype = C.c_void_p
    libc.malloc.argtypes = [C.c_size_t]
    libc.free.argtypes = [C.c_void_p]
    libc.posix_memalign.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_size_t]
    libc.madvise.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    MADV_HUGEPAGE = 14
    nbytes = W * n * 16
    ctxs = [zkl_hip.Context(device) for _ in range(2)]
    src = C.addressof(trace)
    res = {}
    try:
        for c in ctxs:
            c.prove_segment(trace, W, n, pi, opts)  # warm (buffers, tables, upload ring)

        def run(mode):
            times = [[] for _ in ctxs]
            phases = {"malloc": [], "fill": [], "call": [], "upload_loop": [], "free": []}
            bufs = [[c.trace_buffer(nbytes, k) for k in (0, 1)] for c in ctxs] if mode == "pinned" else None

            def work(k):
                for j in range(steps):
                    t0 = time.perf_counter()
                    if mode == "pinned":
                        p = bufs[k][j % 2]
                    elif mode == "thp":
                        q = C.c_void_p()
                        if libc.posix_memalign(C.byref(q), 1 << 21, nbytes):
                            raise MemoryError("posix_memalign of the host trace failed")
                        p = q.value
                        libc.madvise(p, nbytes, MADV_HUGEPAGE)
                    else:
                        p = libc.malloc(nbytes)
                        if not p:
                            raise MemoryError("malloc of the host trace failed")
                    t1 = time.perf_counter()
                    C.memmove(p, src, nbytes)
                    t2 = time.perf_counter()
                    ctxs[k].prove_segment(p, W, n, pi, opts)
                    t3 = time.perf_counter()
                    up = ctxs[k].host_times().get("upload", 0.0)
                    if mode != "pinned":
                        libc.free(p)
                    t4 = time.perf_counter()
                    times[k].append((t4 - t0) * 1e3)
                    for key, v in (("malloc", t1 - t0), ("fill", t2 - t1), ("call", t3 - t2), ("free", t4 - t3)):
                        phases[key].append(v * 1e3)
                    phases["upload_loop"].append(up)
            th = [threading.Thread(target=work, args=(k,)) for k in range(len(ctxs))]
            t0 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            dt = time.perf_counter() - t0
            flat = sorted(t for ts in times for t in ts)
            med = flat[len(flat) // 2]
            return {"value": round(len(flat) / dt, 4), "unit": "segment-proofs/s",
                    "ms_per_proof_call_median": round(med, 2), "max_over_median": round(flat[-1] / med, 3),
                    "phase_ms_median": {k: round(sorted(v)[len(v) // 2], 2) for k, v in phases.items()},
                    "ms_each": [[round(t, 1) for t in ts] for ts in times]}

        res["fresh_malloc"] = run("fresh")
        res["fresh_malloc_hugepages"] = run("thp")
        res["pinned_trace_buffer"] = run("pinned")
    finally:
        for c in ctxs:
            c.close()
    res["note"] = ("2 contexts in flight; each proof's time includes filling the host trace (a 214 MB copy) "
                   "and its upload inside zkl_hip_prove_segment")
    return res


def step_info(zkl_hip, pi, index, total):
    """zl1 step metadata of segment `index` of `total`; the synthetic boundary chain is
    state_out(i) = state_in(i+1) = i+1 (what the aggregation checks)."""
    info = zkl_hip.StepInfo()
    info.suite_id[:] = bytes(pi.program_id)
    info.lambda_bits, info.segment_index, info.segments_total = 128, index, total
    info.state_in_hash[:] = index.to_bytes(32, "little")
    info.state_out_hash[:] = (index + 1).to_bytes(32, "little")
    return info


def handoff(zkl_hip, dist, items, total, chained=False, device=0):
    """Aggregation hand-off: each rank wraps its proofs as zl1 steps (ZKLSTP1),
    rank 0 gathers them over RCCL (zkl_comm_gather_bytes: lengths all-gathered, then one
    ncclSend per rank to the root over xGMI), orders and chain-checks them and forms the
    children root the aggregation proof commits to (agg/child.rs:853-895).  If RCCL cannot
    start on every rank the gather runs over gloo and the line says why.  Returns (summary,
    ordered step bytes) on rank 0."""
    comm, cerr = dist.init_rccl(device)
    t_h = time.perf_counter()
    enc = [chain_step(zkl_hip, i, total, pi, proof) if chained else
           zkl_hip.step_proof_encode(pi, step_info(zkl_hip, pi, i, total), proof) for i, pi, proof in items]
    steps = dist.collect_step_proofs(enc, comm)
    if steps is None:
        return None, None
    root = zkl_hip.children_root(bytes(steps[0]["program_id"]), [d["digest"] for d in steps],
                                 [d["root_trace"] for d in steps])
    out = {"segments": len(steps), "step_bytes": sum(d["bytes"] for d in steps),
           "ms": round((time.perf_counter() - t_h) * 1e3, 2), "children_root": root[:16].hex()}
    if comm is not None:
        out["transport"] = "rccl (ncclAllGather of lengths + ncclSend/ncclRecv to rank 0)"
        out["rccl_device_ms"] = round(comm.last_ms(), 3)
    else:
        out["transport"] = f"gloo ({cerr})"
    return out, [d["raw"] for d in steps]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--cpu-sample-log-n", type=int, default=0,
                    help="rows (log2) of the oracle proof timed for cpu_baseline (0: the headline size, measured)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="oracle threads (0: OMP_NUM_THREADS or min(16, CPUs))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c3-segments", type=int, default=8, help="segments for the configs[2] pipeline line (0: skip)")
    ap.add_argument("--c3-inflight", type=str, default="1,2,4", help="contexts in flight to try for configs[2]")
    ap.add_argument("--segments", type=int, default=-1,
                    help="configs[3] shape: distinct segments sharded over the ranks (-1: 8 x N when N > 1, else 0)")
    ap.add_argument("--inflight", type=int, default=4, help="contexts in flight per rank for --segments")
    ap.add_argument("--c5-log-n", type=int, default=20, help="rows (log2) of the configs[4] single-segment line (0: skip)")
    ap.add_argument("--program-steps", type=int, default=5,
                    help="proofs of the real rollup-bench.zlisp 65,536-row segment (N = 1; 0: skip)")
    ap.add_argument("--host-steps", type=int, default=5,
                    help="proofs timed through zkl_hip_prove_segment with a host-resident trace (N = 1; 0: skip)")
    ap.add_argument("--programs", default="fib-2pow16:65536,rollup-bench:1024",
                    help="real example programs proved segment by segment, sharded over the ranks "
                         "(name:max_segment_rows,...; 'none' to skip)")
    ap.add_argument("--program-inflight", type=int, default=4, help="contexts in flight per rank for --programs")
    ap.add_argument("--tuning", default="spin,malloc",
                    help="opt-in process settings this process applies (zkl_hip_process_tuning): spin, malloc, none")
    ap.add_argument("--dry-run", action="store_true", help="launcher / rank plumbing only, no device work (CPU tests)")
    args = ap.parse_args()
    if args.gpus < 1:
        log("bench: --gpus must be >= 1")
        return 2
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)

    from zkl_hip import dist
    rank, world, local_rank = dist.env()
    if world != args.gpus:
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
            f"(torch.distributed.run --nproc-per-node {args.gpus}) or omit WORLD_SIZE to let bench.py start them")
        return 2

    # Only the result line goes to stdout: native libraries (gloo prints "[Gloo] Rank ..."
    # from C++) write to fd 1, so fd 1 is pointed at stderr and the JSON line is written
    # to a saved copy of the original stdout.
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    dist.init()  # gloo control plane only (zkl_hip/dist.py)
    n_seg = args.segments if args.segments >= 0 else (8 * world if world > 1 else 0)

    if args.dry_run:
        dist.barrier()
        t0 = time.perf_counter()
        dist.barrier()
        elapsed = dist.max_over_ranks(time.perf_counter() - t0)
        mine = dist.segments_for_rank(n_seg, rank, world)
        got = dist.gather_to_root({"rank": rank, "segments": mine, "lines": lines_for_rank(args, world)})
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "dry_run": True,
                              "elapsed_s": elapsed, "segments_by_rank": {g["rank"]: g["segments"] for g in got},
                              "lines_by_rank": {g["rank"]: g["lines"] for g in got},
                              "rccl_required": dist.rccl_required()}),
                  file=result_out, flush=True)
        dist.shutdown()
        return 0

    import zkl_hip
    pinned = os.environ.get("ZKL_BENCH_DEVICE")
    device = int(pinned) if pinned is not None else local_rank
    n_dev = zkl_hip.device_count()
    if device >= n_dev:
        log(f"bench: rank {rank} needs device {device} but {n_dev} HIP device(s) are visible "
            f"(set ZKL_BENCH_DEVICE to rehearse {world} ranks on fewer GPUs)")
        return 3
    want = {x for x in args.tuning.split(",") if x and x != "none"}
    tuning = zkl_hip.process_tuning(spin="spin" in want, malloc="malloc" in want)  # before the first context
    ctx = zkl_hip.Context(device)
    log_n = args.log_n
    n = 1 << log_n
    seed = SEED0 + rank
    trace, pi, W = zkl_hip.synth_vm_segment(seed, log_n)
    opts = zkl_hip.proof_options(W, n)
    nbytes = W * n * 16
    d_trace = ctx.alloc(nbytes)
    ctx.upload(d_trace, trace, nbytes)
    log(f"[rank {rank}] device {device}: trace {W}x{n} resident in HBM; warmup {args.warmup}")

    proof = None
    for _ in range(args.warmup):
        proof = ctx.prove_segment_device(d_trace, W, n, pi, opts)

    kacc = {}
    # every timed proof is written in full into one host buffer kept across steps
    # (zkl_hip_prove_segment_device_into: no per-proof allocation or extra copy on the host side)
    pbuf = bytearray(len(proof) + (1 << 16) if proof else 1 << 20)
    plen = 0
    dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    step_ms, step_stages = [], []
    for i in range(args.steps):
        plen = ctx.prove_segment_device_into(d_trace, W, n, pi, opts, pbuf)
        step_ms.append(ctx.host_times()["call"])
        if os.environ.get("ZKL_BENCH_STAGES"):
            step_stages.append({k: round(v, 2) for k, v in ctx.stage_times().items()})
        for k, (ms, cnt) in ctx.kernel_times().items():
            a = kacc.setdefault(k, [0.0, 0])
            a[0] += ms
            a[1] += cnt
    ctx.synchronize()
    dist.barrier()
    elapsed = dist.max_over_ranks(time.perf_counter() - t0)
    if args.steps:
        proof = bytes(pbuf[:plen])  # the last timed proof, checked below
    host = ctx.host_times()
    parity = dist.gather_to_root(parity_of(proof, seed, log_n))
    stages, fam = {}, {}
    # Inside the timed region only the dominant family (the trace row hash) is bracketed by
    # HIP events (each bracket costs ~10 us of queue time); one extra untimed proof with
    # every family bracketed gives the per-family breakdown.
    if rank == 0:
        ctx.set_kernel_timing(2)
        ctx.prove_segment_device(d_trace, W, n, pi, opts)
        fam = ctx.kernel_times()
        stages = ctx.stage_times()
        ctx.set_kernel_timing(1)
    ctx.free(d_trace)
    # the integration entry point: zkl_hip_prove_segment with the trace in pageable host memory,
    # as the Rust binding passes its Vec; the upload is part of every proof
    host_line = None
    if world == 1 and args.host_steps > 0:
        hp = ctx.prove_segment(trace, W, n, pi, opts)
        ctx.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.host_steps):
            hp = ctx.prove_segment(trace, W, n, pi, opts)
        ctx.synchronize()
        dth = time.perf_counter() - t1
        inflight2 = host_inflight(zkl_hip, device, trace, W, n, pi, opts, args.host_steps)
        fresh = host_fresh(zkl_hip, device, trace, W, n, pi, opts, max(4, args.host_steps))
        host_line = {"entry": "zkl_hip_prove_segment (trace in pageable host memory, uploaded inside each proof)",
                     "value": round(args.host_steps / dth, 4), "unit": "segment-proofs/s",
                     "ms_per_proof": round(dth / args.host_steps * 1e3, 3), "steps": args.host_steps,
                     "trace_bytes": nbytes, "upload_loop_ms_last_proof": round(ctx.host_times().get("upload", 0.0), 3),
                     "parity": parity_of(hp, seed, log_n)["golden"], "two_contexts_in_flight": inflight2,
                     "per_proof_allocation": fresh}
    del trace
    ctx.close()
    hand, _ = handoff(zkl_hip, dist, [(rank, pi, proof)], world, device=device)

    # configs[3] shape: S distinct segments sharded over the ranks, pipelined per rank
    c4 = None
    failures = []  # any golden mismatch or failed line: parity.status MISMATCH and exit code 1
    if n_seg > 0:
        mine = dist.segments_for_rank(n_seg, rank, world)
        pl = Pipeline(zkl_hip, device, log_n, mine, max(1, min(args.inflight, len(mine))))
        dist.barrier()
        t1 = time.perf_counter()
        pl.run()
        dist.barrier()
        el4 = dist.max_over_ranks(time.perf_counter() - t1)
        items = pl.proofs()
        par4 = dist.gather_to_root([chain_parity(i, p) for i, _, p in items])
        pl.close()
        h4, steps4 = handoff(zkl_hip, dist, items, n_seg, chained=True, device=device)
        if rank == 0:
            flat = [g for r in par4 for g in r]
            c4 = {"config": f"BASELINE configs[3] shape: a {n_seg}-segment synthetic program (2^{log_n}-row segments, "
                            f"ROM and VM-state chains) sharded over {world} rank(s), {args.inflight} contexts in flight "
                            "per rank, then the step-proof gather, children root and aggregation proof on rank 0",
                  "value": round(n_seg / el4, 4), "unit": "segment-proofs/s", "seconds": round(el4, 3),
                  "golden_matches": flat.count("match"), "golden_mismatches": flat.count("MISMATCH"),
                  "handoff": h4}
            try:
                c4["aggregation"] = aggregate(zkl_hip, steps4)
            except Exception as e:  # reported in the line, and the run exits non-zero
                c4["aggregation"] = {"error": str(e)}
            if c4["golden_mismatches"] or "error" in c4["aggregation"] or c4["aggregation"].get("golden") == "MISMATCH":
                failures.append("c4_sharded")

    # configs[4]: one 2^20-row segment per rank (replicas), timed between barriers
    c5 = None
    if args.c5_log_n > 0:
        dist.barrier()
        ms5, pb5, err5 = c5_single(zkl_hip, device, args.c5_log_n, barrier=dist.barrier, seed=0x5EED0C05 + rank)
        if err5 is not None:
            err5 = f"rank {rank}: {err5}"
            log(err5)
        errs5 = [e for e in (dist.gather_to_root(err5) or []) if e]
        ms5 = dist.max_over_ranks(ms5 if ms5 is not None else float("inf"))
        if rank == 0:
            if errs5:
                c5 = {"error": "; ".join(errs5)}
            else:
                c5 = {"config": f"BASELINE configs[4] shape: one synthetic 2^{args.c5_log_n}-row segment per rank "
                                f"(blowup 16, q 64, grind 16, partitions (16,16)) on {world} GPU(s): replicas, "
                                "each rank its own segment, max-over-ranks time",
                      "value": round(world / (ms5 * 1e-3), 4), "unit": "segment-proofs/s",
                      "ms_per_proof": round(ms5, 1), "proof_bytes": pb5,
                      "rows_per_s": round(world * (1 << args.c5_log_n) / ms5 * 1e3)}

    # real example programs, segment by segment, sharded over the ranks
    prog_lines = {}
    builders = max(2, cpu_threads(args.cpu_threads) // world)
    for spec in program_specs(args):
        name, mr = spec.split(":")
        pl_out = program_sharded(zkl_hip, dist, device, rank, world, name, int(mr), args.program_inflight,
                                 builders, resident=(name == "fib-2pow16"))
        if rank == 0:
            prog_lines[spec] = pl_out

    # per-rank host footprint and wall time (capacity of N ranks on one host)
    import resource
    pin_now, pin_peak = zkl_hip.pinned_bytes()
    ranks_host = dist.gather_to_root({"rank": rank, "device": device, "wall_s": round(time.time() - T_START, 1),
                                      "max_rss_mb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024),
                                      "pinned_peak_mb": round(pin_peak / 2**20), "pinned_now_mb": round(pin_now / 2**20)})

    if rank == 0:
        value = world * args.steps / elapsed
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
        mism = sum(p["golden"] == "MISMATCH" for p in parity)
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
                "devices": "all ranks pinned to device " + pinned if pinned is not None else "one per rank",
                "proof_bytes": len(proof),
            },
            "parity": {"status": "ok" if mism == 0 and all(p["golden"] == "match" for p in parity)
                       else ("MISMATCH" if mism else "no golden for some ranks"),
                       "reference": "CPU oracle proof bytes (tests/golden/proof_2p16.json)",
                       "ranks": parity},
            "roofline": {
                "bound": "hbm",
                "kernel": f"{kname} (trace LDE row hashing, 4 partitions + merge_many)",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": load_traffic(kname),
                "alg_bytes_per_launch": alg_bytes,
                "avg_launch_ms": round(per_launch_ms, 3),
                "note": "VALU-issue bound (integer Poseidon); see roofline_valu",
            },
            "roofline_valu": valu_roofline(perms_per_s),
            "dominant_kernel_family": dom,
            "kernel_ms_per_family_untimed_step": {k: round(v[0], 3) for k, v in fam.items()},
            "kernel_launches_per_family_untimed_step": {k: v[1] for k, v in fam.items()},
            "stage_ms_untimed_step": {k: round(v, 3) for k, v in stages.items()},
            "host_ms_last_step": {k: round(v, 3) for k, v in host.items()},
            "call_ms_each_step": [round(v, 2) for v in step_ms],
            # stalled-step check: slowest step over the median step
            "max_over_median_step": round(max(step_ms) / sorted(step_ms)[len(step_ms) // 2], 3) if step_ms else None,
            **({"stage_ms_each_step": step_stages} if step_stages else {}),
            "step_handoff": hand,
        }
        if c4 is not None:
            out["c4_sharded"] = c4
        if host_line is not None:
            host_line["fraction_of_resident_rate"] = round(host_line["value"] / value, 4)
            out["host_trace"] = host_line
            if host_line["parity"] == "MISMATCH":
                failures.append("host_trace")
        if world == 1 and args.c3_segments > 0:
            c3 = {}
            for k in [int(x) for x in args.c3_inflight.split(",") if x]:
                pl = Pipeline(zkl_hip, device, log_n, list(range(args.c3_segments)), k)
                best = None
                for _ in range(2):
                    t1 = time.perf_counter()
                    pl.run()
                    dt = time.perf_counter() - t1
                    best = dt if best is None else min(best, dt)
                if k == max(int(x) for x in args.c3_inflight.split(",") if x):
                    g = [chain_parity(i, p) for i, _, p in pl.proofs()]
                    c3_par = {"golden_matches": g.count("match"), "golden_mismatches": g.count("MISMATCH")}
                    c3_steps = [chain_step(zkl_hip, i, args.c3_segments, spi, p) for i, spi, p in pl.proofs()]
                pl.close()
                c3[str(k)] = round(args.c3_segments / best, 4)
            kbest = max(c3, key=lambda k: c3[k])
            out["c3_in_gpu_pipeline"] = {
                "config": f"BASELINE configs[2] shape: the first {args.c3_segments} segments of a synthetic "
                          f"multi-segment program (2^{log_n} rows each) on 1 GPU",
                "segment_proofs_per_s_by_inflight": c3, "best_inflight": int(kbest), "value": c3[kbest],
                "unit": "segment-proofs/s", "parity": c3_par}
            try:
                out["c3_in_gpu_pipeline"]["aggregation"] = aggregate(zkl_hip, c3_steps)
            except Exception as e:  # reported in the line, and the run exits non-zero
                out["c3_in_gpu_pipeline"]["aggregation"] = {"error": str(e)}
            a3 = out["c3_in_gpu_pipeline"]["aggregation"]
            if c3_par["golden_mismatches"] or "error" in a3 or a3.get("golden") == "MISMATCH":
                failures.append("c3_in_gpu_pipeline")
        if c5 is not None:
            out["c5_single_segment"] = c5
            if "error" in c5:
                failures.append("c5_single_segment")
        if prog_lines:
            out["programs"] = prog_lines
            for spec, pl_out in prog_lines.items():
                if "error" in pl_out or pl_out.get("golden_mismatches") or "error" in pl_out.get("aggregation", {}) \
                        or pl_out.get("aggregation", {}).get("golden") == "MISMATCH":
                    failures.append(f"program {spec}")
        out["process_tuning"] = tuning
        out["ranks_host"] = ranks_host
        if world == 1 and args.program_steps > 0:
            try:
                out["real_program"] = real_program(zkl_hip, device, args.program_steps)
                if out["real_program"]["parity"] != "match":
                    failures.append("real_program")
            except Exception as e:  # reported in the line, and the run exits non-zero
                out["real_program"] = {"error": str(e)}
                failures.append("real_program")
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args.cpu_sample_log_n or log_n, cpu_threads(args.cpu_threads),
                                                   proof, log_n)
                if out["cpu_baseline"].get("proof_equals_gpu_proof") is False:
                    failures.append("cpu_baseline proof != GPU proof")
            except Exception as e:  # reported in the line, and the run exits non-zero
                out["cpu_baseline"] = {"value": None, "error": str(e)}
                failures.append("cpu_baseline")
        if out["parity"]["status"] != "ok":
            failures.append("headline parity")
        if failures:
            out["parity"]["status"] = "MISMATCH"
            out["parity"]["failed_lines"] = failures
        print(json.dumps(out), file=result_out, flush=True)
    dist.shutdown()
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
