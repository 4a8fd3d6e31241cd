"""§8(e) multi-rank hand-off, executed: zkl_comm_gather_bytes at world sizes 2 and 3 on one GPU
through a test-only NCCL-ABI library over shared memory (tests/stub/nccl_shm_stub.cpp, selected
with ZKL_RCCL_LIB; real RCCL refuses several ranks on one device).  Covers the branches of
csrc/comm.cpp that a single-GPU run never reaches: the root's ncclRecv loop over its peers, the
non-root ncclSend, a zero-length rank, unequal lengths, capacity growth of the device buffer, a
non-zero root, an all-empty gather, and a failing collective, which must mark the communicator
broken and fail every rank (tests/comm_stub_worker.py runs the ranks)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "stub", "libnccl_shm_stub.so")
WORKER = os.path.join(ROOT, "tests", "comm_stub_worker.py")


def _env(**extra):
    env = dict(os.environ, ZKL_RCCL_LIB=STUB)
    env.update(extra)
    return env


def _py(code, **extra):
    """Runs `code` in a fresh interpreter (comm.cpp opens the NCCL library once per process)."""
    return subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); " % os.path.join(ROOT, "zk-lisp_amd")
                           + code], env=_env(**extra), capture_output=True, text=True, timeout=120)


def test_stub_exports_the_nccl_abi_comm_cpp_binds():
    import ctypes as C
    lib = C.CDLL(STUB)
    for sym in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclAllGather", "ncclSend", "ncclRecv",
                "ncclGroupStart", "ncclGroupEnd", "ncclGetErrorString"):
        assert hasattr(lib, sym), sym


def test_rccl_library_override():
    """ZKL_RCCL_LIB selects the library comm.cpp opens (no device needed to open it and draw a
    unique id); a missing library is reported, not crashed on."""
    r = _py("import zkl_hip; print(zkl_hip.comm_available()); print(zkl_hip.comm_unique_id()[:15])")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "None" and "zkl_nccl_stub_" in lines[1]
    r = _py("import zkl_hip; print(zkl_hip.comm_available())", ZKL_RCCL_LIB="/nonexistent/librccl.so")
    assert r.returncode == 0 and "RCCL not available" in r.stdout


def _ranks(scenario, world, **extra):
    r = _py("import zkl_hip; print(zkl_hip.comm_unique_id().hex())")
    assert r.returncode == 0, r.stderr
    uid = r.stdout.strip()
    procs = [subprocess.Popen([sys.executable, WORKER, scenario, str(k), str(world), uid], env=_env(**extra),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for k in range(world)]
    out = []
    for p in procs:
        so, se = p.communicate(timeout=240)
        out.append((p.returncode, so, se))
    return out


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_gather_branches_multi_rank(world):
    """Four gathers per run: lengths [1000, 0, 3000] to root 0, [10, 5 MiB, 1] (the device buffer
    grows), [200, 300, 0] to root 1, all empty; every root gets every rank's bytes in rank order."""
    res = _ranks("branches", world)
    for rc, so, se in res:
        assert rc == 0, (rc, so, se[-2000:])
    lines = [json.loads(so.strip().splitlines()[-1]) for _, so, _ in res]
    for ln in lines:
        assert all(r["ok"] for r in ln["rounds"]), ln
    root0 = next(ln for ln in lines if ln["rank"] == 0)
    assert root0["rounds"][0]["lens"] == ([1000, 0, 3000][:world])
    assert root0["rounds"][1]["lens"] == ([10, 5 << 20, 1][:world])


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("op,rank,want", [("send", 1, (7, 7)), ("allgather", 0, (7, 7)), ("recv", 0, (7, 0))])
def test_failed_collective_breaks_the_communicator(op, rank, want):
    """An injected fault in one rank's send / all-gather / receive: that rank's gather fails at
    once and its communicator is marked broken (a second gather is refused, exit 7).  A peer that
    waits on the failed rank (the root on a sender that never sent; either rank in the length
    all-gather) fails when its wait runs out, broken as well.  A sender whose blob was delivered
    before the root's receive failed completes (exit 0): the run still fails, on the root, and the
    bench's error flag is reduced over the ranks (bench.py program_sharded)."""
    res = _ranks("fail", 2, ZKL_NCCL_STUB_FAIL=op, ZKL_NCCL_STUB_FAIL_RANK=str(rank), ZKL_NCCL_STUB_TIMEOUT_S="5")
    assert tuple(rc for rc, _, _ in res) == want, [(rc, so, se[-1500:]) for rc, so, se in res]
    msgs = [json.loads(so.strip().splitlines()[-1]) for _, so, _ in res]
    assert "injected" in (msgs[rank]["first"] or "")
