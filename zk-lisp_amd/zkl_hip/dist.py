"""Multi-GPU coordination for segment proving.

Segments are independent, so ranks (one process per GPU, launched by
torch.distributed.run) prove disjoint segment sets with no data-path collective.  The one
exchange is the aggregation hand-off: the step proofs (and the boundary fields inside them)
go to rank 0 over RCCL point-to-point transfers between the GPUs (zkl_comm_*, xGMI within a
node); with one GPU per rank that transport is required (a failure ends the run non-zero), and
gloo carries the bytes only in same-device rehearsals or with ZKL_COMM=gloo, labelled as such.  Control -- the barrier around the timed region, the max-over-ranks elapsed time, the
RCCL unique id -- runs on torch.distributed's gloo backend with CPU tensors: the prover owns
the GPU through its own HIP runtime (runtime note)."""
import os
import struct

_dist = None
_comm = None
_comm_error = None


def env():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init():
    """Join the process group when world_size > 1 (gloo); returns (rank, world, local_rank)."""
    global _dist
    rank, world, local = env()
    if world > 1 and _dist is None:
        import torch.distributed as dist
        if not dist.is_initialized():
            dist.init_process_group("gloo")
        _dist = dist
    return rank, world, local


def segments_for_rank(n_segments, rank, world, rows=None):
    """Segment ids proved by `rank`: greedy by rows (largest first onto the least-loaded
    rank) when per-segment row counts are given, else round-robin i mod world."""
    if rows is None:
        return [i for i in range(n_segments) if i % world == rank]
    load = [0] * world
    owner = [0] * n_segments
    for i in sorted(range(n_segments), key=lambda i: (-rows[i], i)):
        r = min(range(world), key=lambda r: (load[r], r))
        owner[i] = r
        load[r] += rows[i]
    return [i for i in range(n_segments) if owner[i] == rank]


def barrier():
    if _dist is not None:
        _dist.barrier()


def max_over_ranks(x):
    if _dist is None:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    _dist.all_reduce(t, op=_dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x):
    if _dist is None:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    _dist.all_reduce(t, op=_dist.ReduceOp.SUM)
    return float(t.item())


def gather_to_root(obj):
    """Gather one picklable object per rank on rank 0 (list in rank order), None elsewhere."""
    if _dist is None:
        return [obj]
    rank = _dist.get_rank()
    out = [None] * _dist.get_world_size() if rank == 0 else None
    _dist.gather_object(obj, out, dst=0)
    return out


def rccl_required():
    """True when the hand-off must run over RCCL: more than one rank, each on its own GPU
    (ZKL_BENCH_DEVICE unset) and no explicit ZKL_COMM=gloo.  Same-device rehearsals
    (ZKL_BENCH_DEVICE pins every rank to one GPU, which RCCL refuses as a duplicate device) and
    the explicit opt-out keep the gloo transport, labelled as such in the bench line; a
    same-device rehearsal with ZKL_RCCL_LIB (the tests' NCCL-ABI stub) runs the RCCL code path."""
    _, world, _ = env()
    return world > 1 and os.environ.get("ZKL_BENCH_DEVICE") is None and os.environ.get("ZKL_COMM", "rccl") != "gloo"


def _watchdog(seconds, what):
    """Ends the process (exit 3) if `what` has not finished within `seconds`: a collective init
    whose peers failed would otherwise block forever.  Returns the timer; cancel() it after."""
    import threading

    def fire():
        import sys
        print(f"zkl_hip.dist: {what} did not finish within {seconds}s; exiting", file=sys.stderr, flush=True)
        os._exit(3)
    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def init_rccl(device, required=None, timeout_s=180.0):
    """The RCCL communicator of this rank (zkl_hip.Comm): rank 0 draws the unique id and the
    gloo control plane broadcasts it.  Returns (comm or None, error or None).  Before the
    collective ncclCommInitRank every rank reports whether it can enter it, so either all ranks
    enter or none does; a watchdog ends a rank whose init blocks (a peer failed inside it).
    When `required` (default: rccl_required()) any failure raises instead of returning the
    error, so a broken RCCL setup on a multi-GPU node fails the run rather than falling back."""
    global _comm, _comm_error
    if required is None:
        required = rccl_required()
    if _comm is not None or _comm_error is not None:
        if required and _comm is None:
            raise RuntimeError(f"RCCL hand-off required but unavailable: {_comm_error}")
        return _comm, _comm_error
    import zkl_hip
    rank, world, _ = env()
    err, uid = None, None
    if os.environ.get("ZKL_COMM", "rccl") == "gloo":
        err = "ZKL_COMM=gloo"
    elif world > 1 and os.environ.get("ZKL_BENCH_DEVICE") is not None and not os.environ.get("ZKL_RCCL_LIB"):
        err = "same-device rehearsal (ZKL_BENCH_DEVICE pins every rank to one GPU; RCCL needs one GPU per rank)"
    # every rank must be able to enter ncclCommInitRank, or none does (it is collective)
    avail = gather_to_root(err or zkl_hip.comm_available())
    if rank == 0:
        err = next((e for e in avail if e), None)
        if err is None:
            try:
                uid = zkl_hip.comm_unique_id()
            except Exception as e:  # noqa: BLE001  (reported in the bench line)
                err = str(e)
    box = [uid, err]
    if _dist is not None:
        _dist.broadcast_object_list(box, src=0)
    uid, err = box
    comm = None
    if err is None:
        wd = _watchdog(timeout_s, "ncclCommInitRank") if world > 1 else None
        try:
            comm = zkl_hip.Comm(device, world, rank, uid)
        except Exception as e:  # noqa: BLE001
            err = str(e)
        finally:
            if wd is not None:
                wd.cancel()
    errs = gather_to_root(err) if _dist is not None else [err]
    if _dist is not None:  # every rank takes the same transport
        flag = [next((e for e in (errs or []) if e), None)] if rank == 0 else [None]
        _dist.broadcast_object_list(flag, src=0)
        err = flag[0]
    if err is not None and comm is not None:
        comm.close()
        comm = None
    _comm, _comm_error = comm, err
    if required and comm is None:
        raise RuntimeError(f"RCCL hand-off required but unavailable: {err}")
    return comm, err


def pack_blobs(blobs):
    """[u32 count][u64 len]*count[bytes...]: one rank's step proofs as one RCCL payload."""
    head = struct.pack("<I", len(blobs)) + b"".join(struct.pack("<Q", len(b)) for b in blobs)
    return head + b"".join(bytes(b) for b in blobs)


def unpack_blobs(buf):
    (k,) = struct.unpack_from("<I", buf, 0)
    lens = struct.unpack_from(f"<{k}Q", buf, 4)
    out, off = [], 4 + 8 * k
    for n in lens:
        out.append(bytes(buf[off:off + n]))
        off += n
    if off != len(buf):
        raise ValueError("malformed step-proof payload")
    return out


def gather_timeout_s():
    """Seconds the RCCL step-proof gather may take once every rank has entered it
    (ZKL_GATHER_TIMEOUT_S, default 300)."""
    return float(os.environ.get("ZKL_GATHER_TIMEOUT_S", "300"))


def gather_step_bytes(step_bytes, comm=None):
    """Every rank's step encodings on rank 0 (list per rank), None elsewhere: over RCCL when a
    communicator is given, else over gloo (host bytes).  The ranks meet at a gloo barrier first,
    so the watchdog times the transfer itself, not a slower rank's proving."""
    if comm is not None:
        _, world, _ = env()
        barrier()
        wd = _watchdog(gather_timeout_s(), "the RCCL step-proof gather") if world > 1 else None
        try:
            got = comm.gather_bytes(pack_blobs(step_bytes), root=0)
        finally:
            if wd is not None:
                wd.cancel()
        return None if got is None else [unpack_blobs(b) for b in got]
    return gather_to_root(list(step_bytes))


def collect_step_proofs(step_bytes, comm=None):
    """Aggregation hand-off: every rank contributes the ZKLSTP1 encodings of
    the step proofs it produced; rank 0 receives all of them, decodes each one
    (StepProof::from_bytes field order, proof/step.rs:153-493), orders them by segment
    index and checks the boundary chain the aggregation AIR consumes (state_out_hash of
    segment i == state_in_hash of segment i+1) and the step digests (digest.rs:16-68).
    Returns the ordered list of dicts on rank 0, None elsewhere.  The payload (~0.47 MB per
    2^16-row segment) moves over RCCL when `comm` is given (gather_step_bytes)."""
    from . import parse_step_proof, step_proof_digest
    got = gather_step_bytes(step_bytes, comm)
    if got is None:
        return None
    steps = []
    for per_rank in got:
        for b in per_rank:
            d = parse_step_proof(b)
            d["digest"], d["root_trace"] = step_proof_digest(b)
            d["bytes"] = len(b)
            d["raw"] = bytes(b)
            steps.append(d)
    steps.sort(key=lambda d: d["segment_index"])
    total = steps[0]["segments_total"] if steps else 0
    if [d["segment_index"] for d in steps] != list(range(len(steps))) or (total > 1 and total != len(steps)):
        raise ValueError("step proofs do not cover segments 0..n-1 exactly once")
    for a, b in zip(steps, steps[1:]):
        if a["state_out_hash"] != b["state_in_hash"]:
            raise ValueError(f"segment {b['segment_index']}: state_in_hash does not continue segment "
                             f"{a['segment_index']}")
    return steps


def shutdown():
    global _dist, _comm, _comm_error
    if _comm is not None:
        _comm.close()
    _comm, _comm_error = None, None
    if _dist is not None:
        _dist.destroy_process_group()
        _dist = None
