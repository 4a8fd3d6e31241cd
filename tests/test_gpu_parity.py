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
    rng = random.Random(5)
    P = oracle.P
    ncols, nrows = 51, 1024
    vals = [rng.randrange(P) for _ in range(ncols * nrows)]
    raw = (C.c_uint8 * (16 * ncols * nrows)).from_buffer_copy(b"".join(v.to_bytes(16, "little") for v in vals))
    d_m = gpu_ctx.alloc(len(raw))
    d_o = gpu_ctx.alloc(nrows * 16)
    d_nodes = gpu_ctx.alloc(2 * nrows * 16)
    gpu_ctx.upload(d_m, raw, len(raw))
    gpu_ctx.hash_rows(d_m, ncols, nrows, 1, 16, d_o)
    got = gpu_ctx.download(d_o, nrows * 16)
    for r in range(0, nrows, 97):
        row = [vals[c * nrows + r] for c in range(ncols)]
        assert int.from_bytes(got[16 * r:16 * r + 16], "little") == oracle.hash_elements(row)
    gpu_ctx.merkle_tree(d_o, nrows, d_nodes)
    nodes = gpu_ctx.download(d_nodes, 2 * nrows * 16)
    lvl = [int.from_bytes(got[16 * i:16 * i + 16], "little") for i in range(nrows)]
    while len(lvl) > 1:
        lvl = [oracle.merge(lvl[2 * i], lvl[2 * i + 1]) for i in range(len(lvl) // 2)]
    assert int.from_bytes(nodes[16:32], "little") == lvl[0]
    for d in (d_m, d_o, d_nodes):
        gpu_ctx.free(d)


def test_stage_lde_matches_oracle(oracle, gpu_ctx):
    """zkl_hip_lde: coefficients and coset LDE (GENERATOR * <w_{16n}>) vs direct evaluation."""
    rng = random.Random(9)
    P = oracle.P
    ncols, n, blow = 3, 64, 16
    N = n * blow
    vals = [rng.randrange(P) for _ in range(ncols * n)]
    raw = (C.c_uint8 * (16 * ncols * n)).from_buffer_copy(b"".join(v.to_bytes(16, "little") for v in vals))
    d_v = gpu_ctx.alloc(len(raw))
    d_c = gpu_ctx.alloc(len(raw))
    d_l = gpu_ctx.alloc(16 * ncols * N)
    gpu_ctx.upload(d_v, raw, len(raw))
    gpu_ctx.lde(d_v, ncols, n, blow, d_c, d_l)
    coef = gpu_ctx.download(d_c, len(raw))
    lde = gpu_ctx.download(d_l, 16 * ncols * N)
    g = oracle.root_of_unity(6)
    w = oracle.root_of_unity(10)
    for c in range(ncols):
        cs = [int.from_bytes(coef[16 * (c * n + k):16 * (c * n + k + 1)], "little") for k in range(n)]
        for r in (0, 5, 63):
            x = pow(g, r, P)
            assert sum(cs[k] * pow(x, k, P) for k in range(n)) % P == vals[c * n + r]
        for i in (0, 1, 17, N - 1):
            x = 3 * pow(w, i, P) % P
            want = sum(cs[k] * pow(x, k, P) for k in range(n)) % P
            assert int.from_bytes(lde[16 * (c * N + i):16 * (c * N + i + 1)], "little") == want
    for d in (d_v, d_c, d_l):
        gpu_ctx.free(d)
