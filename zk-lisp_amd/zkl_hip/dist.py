"""Multi-GPU coordination for segment proving.

Segments are independent, so ranks (one process per GPU, launched by
torch.distributed.run) prove disjoint segment sets with no data-path collective.  The
only communication is control: a barrier around the timed region, the max-over-ranks
elapsed time, and (for the aggregation hand-off) gathering step-proof bytes on rank 0.
It runs on torch.distributed's gloo backend with CPU tensors: the prover owns the GPU
through its own HIP runtime (runtime note)."""
import os

_dist = None


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


def collect_step_proofs(step_bytes):
    """Aggregation hand-off: every rank contributes the ZKLSTP1 encodings of
    the step proofs it produced; rank 0 receives all of them, decodes each one
    (StepProof::from_bytes field order, proof/step.rs:153-493), orders them by segment
    index and checks the boundary chain the aggregation AIR consumes (state_out_hash of
    segment i == state_in_hash of segment i+1) and the step digests (digest.rs:16-68).
    Returns the ordered list of dicts on rank 0, None elsewhere.  The payload is a few
    hundred KB per segment, so it travels over the gloo control plane as host bytes."""
    from . import parse_step_proof, step_proof_digest
    got = gather_to_root(list(step_bytes))
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
    global _dist
    if _dist is not None:
        _dist.destroy_process_group()
        _dist = None
