"""GPU parity: libzkl_hip.so proofs are byte-identical to the CPU oracle's on the same
inputs; stage entry points agree with the oracle; full-size proofs are deterministic."""
import ctypes as C
import hashlib
import random

import pytest

pytestmark = pytest.mark.gpu


def _pi_copy(src, cls):
    dst = cls()
    C.memmove(C.byref(dst), C.byref(src), C.sizeof(dst))
    return dst


def _gpu_opts(zkl_hip, o):
    return zkl_hip.ProofOptions(*[getattr(o, f) for f, _ in o._fields_])


@pytest.mark.parametrize("log_n,q,blowup,grind", [
    (5, 8, 16, 0), (5, 64, 16, 8), (6, 32, 8, 4), (8, 64, 16, 10), (10, 64, 16, 12), (9, 20, 32, 6),
])
def test_proof_bytes_match_oracle(oracle, gpu_ctx, log_n, q, blowup, grind):
    import zkl_hip
    n = 1 << log_n
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0001 + log_n, log_n)
    opts = zkl_hip.proof_options(w, n, queries=q, blowup=blowup, grind=grind)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    ot, opi, _ = oracle.synth_segment(0x5EED0001 + log_n, log_n)
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    want = oracle.prove(ot, w, n, opi, oo)
    assert len(got) == len(want)
    assert got == want


def test_multi_partition_parity(oracle, gpu_ctx):
    """n = 2^14 exercises 2-way row partitioning + merge_many (PartitionOptions)."""
    import zkl_hip
    oracle.set_threads(16)
    n = 1 << 14
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0100, 14)
    opts = zkl_hip.proof_options(w, n, queries=32, grind=8)
    assert opts.num_partitions == 2
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    ot, opi, _ = oracle.synth_segment(0x5EED0100, 14)
    want = oracle.prove(ot, w, n, opi, oo)
    oracle.set_threads(1)
    assert got == want


def test_invalid_trace_rejected(gpu_ctx):
    import zkl_hip
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0001, 6)
    t[(42 + 3) * 64 + 40].lo ^= 1
    opts = zkl_hip.proof_options(w, 64, queries=8, grind=0)
    with pytest.raises(zkl_hip.ZklError, match="degree too large"):
        gpu_ctx.prove_segment(t, w, 64, pi, opts)


def test_full_size_deterministic(gpu_ctx):
    """BASELINE config: 65536 rows, blowup 16, q 64, grind 16; two runs, same bytes."""
    import zkl_hip
    n = 1 << 16
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0001, 16)
    opts = zkl_hip.proof_options(w, n)
    assert (opts.num_partitions, opts.hash_rate) == (4, 16)
    a = gpu_ctx.prove_segment(t, w, n, pi, opts)
    b = gpu_ctx.prove_segment(t, w, n, pi, opts)
    assert a == b
    print("full-size proof", len(a), hashlib.sha256(a).hexdigest(), gpu_ctx.stage_times())


def test_stage_hash_rows_and_merkle(oracle, gpu_ctx):
    import torch
    rng = random.Random(5)
    P = oracle.P
    ncols, nrows = 51, 1024
    vals = [rng.randrange(P) for _ in range(ncols * nrows)]
    raw = b"".join(v.to_bytes(16, "little") for v in vals)
    d_m = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    d_o = torch.zeros(nrows * 16, dtype=torch.uint8, device="cuda")
    gpu_ctx.hash_rows(d_m.data_ptr(), ncols, nrows, 1, 16, d_o.data_ptr())
    torch.cuda.synchronize()
    got = bytes(d_o.cpu().numpy().tobytes())
    for r in range(0, nrows, 97):
        row = [vals[c * nrows + r] for c in range(ncols)]
        assert int.from_bytes(got[16 * r:16 * r + 16], "little") == oracle.hash_elements(row)
    d_nodes = torch.zeros(2 * nrows * 16, dtype=torch.uint8, device="cuda")
    gpu_ctx.merkle_tree(d_o.data_ptr(), nrows, d_nodes.data_ptr())
    torch.cuda.synchronize()
    nodes = bytes(d_nodes.cpu().numpy().tobytes())
    leaves = [int.from_bytes(got[16 * i:16 * i + 16], "little") for i in range(nrows)]
    lvl = leaves
    while len(lvl) > 1:
        lvl = [oracle.merge(lvl[2 * i], lvl[2 * i + 1]) for i in range(len(lvl) // 2)]
    assert int.from_bytes(nodes[16:32], "little") == lvl[0]
