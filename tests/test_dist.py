"""World-size-2 gloo tests (CPU) of the multi-GPU coordination used by bench.py:
segment sharding, barrier, max/sum over ranks and the step-proof gather to rank 0."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_segment_assignment_partitions_work():
    sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))
    from zkl_hip import dist
    for world in (1, 2, 3, 8):
        got = sorted(i for r in range(world) for i in dist.segments_for_rank(64, r, world))
        assert got == list(range(64))
        assert all(len(dist.segments_for_rank(64, r, world)) in (64 // world, 64 // world + 1) for r in range(world))
    rows = [65536] * 6 + [4096] * 10
    per = [dist.segments_for_rank(16, r, 4, rows) for r in range(4)]
    assert sorted(i for p in per for i in p) == list(range(16))
    loads = [sum(rows[i] for i in p) for p in per]
    assert max(loads) - min(loads) <= 65536


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))
    from zkl_hip import dist
    r, w, lr = dist.init()
    dist.barrier()
    mx = dist.max_over_ranks(1.5 + r)
    sm = dist.sum_over_ranks(r + 1)
    mine = dist.segments_for_rank(8, r, w)
    g = dist.gather_to_root({"rank": r, "segments": mine, "proof": bytes([r]) * (r + 3)})
    q.put((r, w, lr, mx, sm, mine, g))
    dist.shutdown()


def _step_worker(rank, world, port, q):
    """Rank r wraps an oracle proof of its own segment as step r of `world` (host-only
    library calls) and hands it to rank 0, as bench.py does after the timed region."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    for p in (os.path.join(ROOT, "zk-lisp_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import ctypes as C
    import oracle_lib
    import zkl_hip
    from zkl_hip import dist
    dist.init()
    # no GPU here: every rank gets the same error, and with required=False gloo carries the bytes
    comm, cerr = dist.init_rccl(0, required=False)
    t, opi, w = oracle_lib.synth_segment(0x5EED7000 + rank, 5)
    inner = oracle_lib.prove(t, w, 32, opi, oracle_lib.default_options(w, 32, queries=4, grind=0))
    pi = zkl_hip.AirPublicInputs()
    C.memmove(C.byref(pi), C.byref(opi), C.sizeof(pi))
    info = zkl_hip.StepInfo()
    info.suite_id[:] = bytes(pi.program_id)
    info.lambda_bits, info.segment_index, info.segments_total = 64, rank, world
    info.state_in_hash[:] = bytes([rank]) * 32       # chained: out(r) = in(r+1)
    info.state_out_hash[:] = bytes([rank + 1]) * 32
    step = zkl_hip.step_proof_encode(pi, info, inner)
    steps = dist.collect_step_proofs([step], comm)
    root = None
    if steps is not None:
        root = zkl_hip.children_root(bytes(pi.program_id), [d["digest"] for d in steps],
                                     [d["root_trace"] for d in steps])
    q.put((rank, None if steps is None else [(d["segment_index"], d["digest"], d["root_trace"]) for d in steps],
           zkl_hip.step_proof_digest(step), root, bytes(pi.program_id), (comm is None, cerr)))
    dist.shutdown()


def test_gloo_step_handoff_world_size_2():
    """World size 2: each rank's step proof reaches rank 0 intact (digest, root_trace),
    ordered by segment, chain-checked, and rank 0 forms the children root over them."""
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))
    import zkl_hip
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_step_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res, transport = {}, {}
    for _ in range(2):
        r, steps, own, root, suite, tr = q.get(timeout=180)
        res[r] = (steps, own, root, suite)
        transport[r] = tr
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # RCCL could not start (no GPU): both ranks fell back together, with the reason
    assert transport[0] == transport[1] and transport[0][0] and transport[0][1]
    steps, _, root, suite = res[0]
    assert res[1][0] is None and res[1][2] is None
    assert [s[0] for s in steps] == [0, 1]
    assert (steps[0][1], steps[0][2]) == res[0][1] and (steps[1][1], steps[1][2]) == res[1][1]
    assert root == zkl_hip.children_root(suite, [s[1] for s in steps], [s[2] for s in steps])
    assert root != bytes(32)


def _required_worker(rank, world, port, q, pinned):
    """init_rccl with the default policy: one GPU per rank (no ZKL_BENCH_DEVICE) requires RCCL,
    so with no GPU every rank raises; a same-device rehearsal falls back to gloo, labelled."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.pop("ZKL_COMM", None)
    if pinned:
        os.environ["ZKL_BENCH_DEVICE"] = "0"
    else:
        os.environ.pop("ZKL_BENCH_DEVICE", None)
    sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))
    from zkl_hip import dist
    dist.init()
    try:
        comm, err = dist.init_rccl(0)
        res = ("fallback", comm is None, err)
    except RuntimeError as e:
        res = ("raised", None, str(e))
    q.put((rank, dist.rccl_required(), res))
    dist.shutdown()


@pytest.mark.parametrize("pinned", [False, True])
def test_rccl_required_with_one_gpu_per_rank(pinned):
    """with one GPU per rank a failed RCCL start raises on every rank (the
    bench then exits non-zero) instead of silently degrading to gloo; a same-device rehearsal
    (ZKL_BENCH_DEVICE) keeps gloo and says so."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_required_worker, args=(r, 2, port, q, pinned)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (req, x)) for r, req, x in (q.get(timeout=180) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        req, (kind, none, msg) = res[r]
        assert req is (not pinned)
        if pinned:
            assert kind == "fallback" and none and "same-device rehearsal" in msg
        else:
            assert kind == "raised" and "RCCL hand-off required" in msg


def test_bench_dry_run_reports_lines_and_transport_policy():
    """--dry-run at N = 2: every rank runs the configs[4] replica line (c5_single_segment) and
    the sharded configs[3] line; the RCCL hand-off is required with one GPU per rank and not in
    a same-device rehearsal."""
    import json
    for env, req in (({}, True), ({"ZKL_BENCH_DEVICE": "0"}, False), ({"ZKL_COMM": "gloo"}, False)):
        r = _bench(["--gpus", "2", "--dry-run"], env)
        assert r.returncode == 0, r.stderr[-2000:]
        out = json.loads(r.stdout.strip().splitlines()[-1])
        assert out["rccl_required"] is req
        for rank in ("0", "1"):
            lines = out["lines_by_rank"][rank]
            assert "c5_single_segment" in lines and "c4_sharded" in lines and "real_program" not in lines
    r = _bench(["--gpus", "1", "--dry-run"])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["rccl_required"] is False and "real_program" in out["lines_by_rank"]["0"]


def test_step_chain_check_rejects_broken_chain():
    """collect_step_proofs (single process: the gather is the identity) rejects a state
    hash that does not continue the previous segment and a missing segment."""
    sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    import oracle_lib
    import zkl_hip
    from zkl_hip import dist
    t, opi, w = oracle_lib.synth_segment(0x5EED7100, 5)
    inner = oracle_lib.prove(t, w, 32, opi, oracle_lib.default_options(w, 32, queries=4, grind=0))
    pi = zkl_hip.AirPublicInputs()
    C.memmove(C.byref(pi), C.byref(opi), C.sizeof(pi))

    def step(i, total, sin, sout):
        info = zkl_hip.StepInfo()
        info.suite_id[:] = bytes(pi.program_id)
        info.segment_index, info.segments_total = i, total
        info.state_in_hash[:] = bytes([sin]) * 32
        info.state_out_hash[:] = bytes([sout]) * 32
        return zkl_hip.step_proof_encode(pi, info, inner)

    ok = dist.collect_step_proofs([step(1, 3, 1, 2), step(0, 3, 0, 1), step(2, 3, 2, 3)])
    assert [d["segment_index"] for d in ok] == [0, 1, 2]
    with pytest.raises(ValueError, match="state_in_hash"):
        dist.collect_step_proofs([step(0, 2, 0, 1), step(1, 2, 5, 6)])
    with pytest.raises(ValueError, match="exactly once"):
        dist.collect_step_proofs([step(0, 3, 0, 1), step(2, 3, 1, 2)])


def test_gloo_world_size_2():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, w, lr, mx, sm, mine, g = q.get(timeout=120)
        res[r] = (w, lr, mx, sm, mine, g)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][2] == res[1][2] == 2.5
    assert res[0][3] == res[1][3] == 3.0
    assert res[0][4] == [0, 2, 4, 6] and res[1][4] == [1, 3, 5, 7]
    g = res[0][5]
    assert [x["rank"] for x in g] == [0, 1] and g[1]["proof"] == b"\x01" * 4
    assert res[1][5] is None


def _bench(args, env_extra=None, timeout=180):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_launcher_spawns_ranks():
    """`bench.py --gpus 2` without a torch.distributed.run environment starts two ranks itself
    (gloo rendezvous on 127.0.0.1), and rank 0's line reports n_gpus 2 with the configs[3]
    segments sharded over both ranks (--dry-run: no device work)."""
    import json
    r = _bench(["--gpus", "2", "--dry-run", "--segments", "16"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["dry_run"]
    seg = out["segments_by_rank"]
    assert sorted(seg["0"] + seg["1"]) == list(range(16)) and seg["0"] == list(range(0, 16, 2))


def test_bench_rejects_world_mismatch():
    """Under a torch.distributed.run environment WORLD_SIZE must equal --gpus (ADVICE r1:
    --gpus was parsed and ignored)."""
    r = _bench(["--gpus", "4", "--dry-run"], {"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def test_bench_launcher_propagates_rank_failure():
    """A failing rank makes the launcher exit non-zero and print no result line."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"ZKL_BENCH_DEVICE": "99"})
    assert r.returncode != 0
    assert r.stdout.strip() == ""


def test_step_blob_packing():
    """One rank's step proofs travel as one RCCL payload: [u32 count][u64 len]*[bytes]."""
    sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))
    from zkl_hip import dist
    for blobs in ([], [b""], [b"a"], [bytes(range(256)) * 3, b"", b"xyz"]):
        assert dist.unpack_blobs(dist.pack_blobs(blobs)) == blobs
    with pytest.raises(ValueError):
        dist.unpack_blobs(dist.pack_blobs([b"abc"]) + b"!")
