"""One rank of tests/test_comm_stub.py (test infrastructure): drives zkl_comm_gather_bytes through
the NCCL-ABI shared-memory stub (ZKL_RCCL_LIB) with several processes on one GPU.

    python tests/comm_stub_worker.py <scenario> <rank> <world> <uid hex>

scenario "branches": four gathers -- unequal lengths with a zero-length rank, a blob larger than
the communicator's buffer (capacity growth), a non-zero root, every rank empty -- each checked on
its root; prints one JSON line; exit 0 / 5 (wrong bytes).
scenario "fail": one gather under the stub's injected fault (ZKL_NCCL_STUB_FAIL); if it raises, a
second one must be refused (the communicator is marked broken): exit 7 then, 6 if the second was not
refused, 0 if the first gather succeeded (a sender whose blob was delivered before the root failed)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-lisp_amd"))
import zkl_hip  # noqa: E402

ROUNDS = [  # (root, per-rank lengths); ranks beyond the list send nothing
    (0, [1000, 0, 3000]),
    (0, [10, 5 << 20, 1]),
    (1, [200, 300, 0]),
    (0, [0, 0, 0]),
]


def payload(rnd, rank, n):
    return bytes((rank * 31 + rnd * 7 + i) % 251 for i in range(n)) if n < 4096 else \
        (bytes([(rank * 31 + rnd * 7) % 251]) * 4096) * (n // 4096) + bytes(n % 4096)


def main():
    scenario, rank, world, uid = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), bytes.fromhex(sys.argv[4])
    comm = zkl_hip.Comm(0, world, rank, uid)
    if scenario == "fail":
        try:
            comm.gather_bytes(b"x" * 100, root=0)
        except zkl_hip.ZklError as e:
            first = str(e)
        else:  # a sender whose blob was delivered before the root failed completes its gather
            print(json.dumps({"rank": rank, "first": None}), flush=True)
            return 0
        try:
            comm.gather_bytes(b"y", root=0)
        except zkl_hip.ZklError as e:
            second = str(e)
        else:
            return 6
        print(json.dumps({"rank": rank, "first": first, "second": second}), flush=True)
        return 7 if "earlier collective" in second else 6
    res = []
    for rnd, (root, lens) in enumerate(ROUNDS):
        lens = (lens + [0] * world)[:world]
        got = comm.gather_bytes(payload(rnd, rank, lens[rank]), root=root)
        if rank == root:
            want = [payload(rnd, r, lens[r]) for r in range(world)]
            res.append({"round": rnd, "ok": got == want, "lens": [len(g) for g in got], "ms": comm.last_ms()})
        else:
            res.append({"round": rnd, "ok": got is None})
    comm.close()
    print(json.dumps({"rank": rank, "rounds": res}), flush=True)
    return 0 if all(r["ok"] for r in res) else 5


if __name__ == "__main__":
    sys.exit(main())
