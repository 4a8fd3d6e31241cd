"""RCCL boundary exchange (zkl_comm_*) on the GPU box.  The box has one GPU,
so the collective runs at world size 1 here (length all-gather, the root's own blob through
the device buffer); the multi-rank path is the same calls with ncclSend / ncclRecv between
GPUs, and its coordination is covered by tests/test_dist.py with gloo at world size 2."""
import os

import pytest

import zkl_hip


def test_comm_symbols_and_cpu_behaviour():
    lib = zkl_hip.load_library()
    for f in ("zkl_comm_available", "zkl_comm_unique_id", "zkl_comm_init", "zkl_comm_gather_bytes",
              "zkl_comm_last_ms", "zkl_comm_destroy"):
        assert hasattr(lib, f)
    assert lib.zkl_comm_init(0, 0, 0, bytes(128), None) != 0  # world 0 rejected before any RCCL call


@pytest.mark.gpu
@pytest.mark.parametrize("size", [0, 1, 4097, 3 << 20])
def test_rccl_gather_world_1(size):
    assert zkl_hip.comm_available() is None
    comm = zkl_hip.Comm(0, 1, 0, zkl_hip.comm_unique_id())
    try:
        data = os.urandom(size)
        got = comm.gather_bytes(data, root=0)
        assert got == [data]
        got = comm.gather_bytes(data[: size // 2], root=0)  # reuses the device buffers
        assert got == [data[: size // 2]]
        assert comm.last_ms() >= 0
    finally:
        comm.close()


@pytest.mark.gpu
def test_rccl_step_proof_handoff_world_1():
    """collect_step_proofs over RCCL returns the step proofs the gloo path returns."""
    from zkl_hip import dist
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED7100, 5)
    info = zkl_hip.step_info_for(pi, 0, 1, bytes(32), bytes([1]) * 32)
    ctx = zkl_hip.Context(0)
    try:
        proof = ctx.prove_segment(t, w, 32, pi, zkl_hip.proof_options(w, 32, queries=8, grind=0))
    finally:
        ctx.close()
    step = zkl_hip.step_proof_encode(pi, info, proof)
    comm = zkl_hip.Comm(0, 1, 0, zkl_hip.comm_unique_id())
    try:
        a = dist.collect_step_proofs([step], comm)
        b = dist.collect_step_proofs([step], None)
        assert [d["raw"] for d in a] == [d["raw"] for d in b] == [step]
    finally:
        comm.close()
