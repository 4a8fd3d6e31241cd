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
