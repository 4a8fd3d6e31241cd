"""GPU parity: libzkl_hip.so proofs are byte-identical to the CPU oracle's on the same
inputs; stage entry points agree with the oracle; full-size proofs are deterministic."""
import ctypes as C
import hashlib
import os
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
    (5, 1, 16, 0),      # a single query
    (5, 255, 8, 2),     # maximum queries on a 256-point domain: heavy position collisions
    (6, 16, 64, 3),     # blowup 64
    (11, 32, 16, 14),   # long grinding search
])
def test_proof_bytes_match_oracle(oracle, gpu_ctx, log_n, q, blowup, grind):
    import zkl_hip
    oracle.set_threads(16 if log_n >= 10 else 1)
    n = 1 << log_n
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0001 + log_n, log_n)
    opts = zkl_hip.proof_options(w, n, queries=q, blowup=blowup, grind=grind)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    ot, opi, _ = oracle.synth_segment(0x5EED0001 + log_n, log_n)
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    want = oracle.prove(ot, w, n, opi, oo)
    assert len(got) == len(want)
    assert got == want
    rc, err = oracle.verify(got, opi, oo)
    assert rc == 0, err


def test_grinding_windows_match_oracle(oracle, gpu_ctx):
    """Grinding queues four ascending nonce windows per read-back (2^g, 2^g, 2^(g+1), 2^(g+2)
    tries) and a window's kernel stops early only for a solution of an EARLIER window: over ten
    seeds at grind 14 some nonces fall past the first window, and every proof (nonce, queries,
    openings) must equal the oracle's sequential search (winterfell without `concurrent`)."""
    import zkl_hip
    oracle.set_threads(1)
    n = 1 << 5
    for k in range(10):
        seed = 0x6B1D0000 + k
        t, pi, w = zkl_hip.synth_vm_segment(seed, 5)
        opts = zkl_hip.proof_options(w, n, queries=8, blowup=16, grind=14)
        got = gpu_ctx.prove_segment(t, w, n, pi, opts)
        ot, opi, _ = oracle.synth_segment(seed, 5)
        want = oracle.prove(ot, w, n, opi, oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_]))
        assert got == want, f"seed {seed:#x}"


@pytest.mark.parametrize("first", [1, 3, 64])
def test_grinding_host_continuation_matches_oracle(oracle, gpu_ctx, monkeypatch, first):
    """when the first four device windows hold no nonce (probability e^-8 at the
    default window size), the host continues the search window by window and derives the query
    seed itself (merge_with_int, prover.cpp).  ZKL_TEST_GRIND_FIRST shrinks the first window to
    `first` tries so the first pass (first * 8 tries) misses at grind 10 and the continuation
    runs; the proof must still equal the oracle's sequential search."""
    import zkl_hip
    oracle.set_threads(1)
    monkeypatch.setenv("ZKL_TEST_GRIND_FIRST", str(first))
    n = 1 << 6
    past = 0
    for k in range(3):
        seed = 0x6B1E0000 + k
        t, pi, w = zkl_hip.synth_vm_segment(seed, 6)
        opts = zkl_hip.proof_options(w, n, queries=16, blowup=16, grind=10)
        got = gpu_ctx.prove_segment(t, w, n, pi, opts)
        ot, opi, _ = oracle.synth_segment(seed, 6)
        want = oracle.prove(ot, w, n, opi, oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_]))
        assert got == want, f"seed {seed:#x}"
        past += int.from_bytes(got[-8:], "little") > first * 8  # Proof::to_bytes ends with the nonce
        zkl_hip.verify_segment(got, pi, opts)
    assert past > 0  # the host continuation found at least one of the nonces


@pytest.mark.parametrize("log_n,q,blowup,grind", [
    (5, 8, 16, 0), (6, 32, 8, 4), (8, 64, 16, 10), (10, 64, 16, 12), (7, 255, 8, 1),
])
def test_sponge_proof_bytes_match_oracle(oracle, gpu_ctx, log_n, q, blowup, grind):
    """Segments with SAbsorbN / SSqueeze enable the Poseidon AIR block (poseidon.rs:26-162):
    27x12 round constraints, 12 hold constraints and the VM->lane bindings (degree 6/3)."""
    import zkl_hip
    oracle.set_threads(16 if log_n >= 10 else 1)
    n = 1 << log_n
    seed = 0x5B0A6E00 + log_n
    t, pi, w = zkl_hip.synth_vm_segment(seed, log_n, 1)
    assert pi.segment_feature_mask == zkl_hip.FM_VM | zkl_hip.FM_SPONGE | zkl_hip.FM_POSEIDON
    opts = zkl_hip.proof_options(w, n, queries=q, blowup=blowup, grind=grind)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    ot, opi, _ = oracle.synth_segment(seed, log_n, 1)
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    want = oracle.prove(ot, w, n, opi, oo)
    oracle.set_threads(1)
    assert got == want
    rc, err = oracle.verify(got, opi, oo)
    assert rc == 0, err


def test_sponge_bad_lane_rejected(gpu_ctx):
    """A Poseidon lane value off its permutation breaks a round constraint."""
    import zkl_hip
    n = 1 << 8
    t, pi, w = zkl_hip.synth_vm_segment(0x5B0A6E08, 8, 1)
    t[3 * n + 32 * 3 + 9].lo ^= 1      # lane 3, round row 8 of level 3 (a squeeze level)
    opts = zkl_hip.proof_options(w, n, queries=8, grind=0)
    with pytest.raises(zkl_hip.ZklError, match="degree too large"):
        gpu_ctx.prove_segment(t, w, n, pi, opts)


def test_sponge_full_size_verifies(oracle, gpu_ctx):
    """configs[1] shape (2^16 rows, blowup 16, q 64, grind 16) with the Poseidon block on."""
    import zkl_hip
    n = 1 << 16
    t, pi, w = zkl_hip.synth_vm_segment(0x5B0A6E10, 16, 1)
    opts = zkl_hip.proof_options(w, n)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    _, opi, _ = oracle.synth_segment(0x5B0A6E10, 16, 1)
    rc, err = oracle.verify(got, opi, oo)
    assert rc == 0, err


@pytest.mark.parametrize("flags,log_n,q,blowup,grind", [
    (2, 8, 32, 16, 4),     # RAM: {vm, ram, rom}, W = 212
    (2, 11, 64, 16, 10),   # RAM with the delta_clk gadget over several bits
    (4, 8, 16, 8, 2),      # Merkle path: {vm, merkle, rom}, W = 211
    (6, 10, 64, 16, 8),    # RAM + Merkle: baseline layout W = 219
    (7, 9, 48, 32, 6),     # sponge + RAM + Merkle
    (3, 12, 64, 16, 12),   # sponge + RAM
])
def test_ram_merkle_proof_bytes_match_oracle(oracle, gpu_ctx, flags, log_n, q, blowup, grind):
    """RamAir (ram.rs:82-236) and MerkleAir (merkle.rs:60-134) blocks on the GPU evaluator."""
    import zkl_hip
    oracle.set_threads(16 if log_n >= 10 else 1)
    n = 1 << log_n
    seed = 0x5EED0500 + 16 * flags + log_n
    t, pi, w = zkl_hip.synth_vm_segment(seed, log_n, flags)
    opts = zkl_hip.proof_options(w, n, queries=q, blowup=blowup, grind=grind)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    ot, opi, _ = oracle.synth_segment(seed, log_n, flags)
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    want = oracle.prove(ot, w, n, opi, oo)
    oracle.set_threads(1)
    assert got == want
    rc, err = oracle.verify(got, opi, oo)
    assert rc == 0, err


def test_ram_merkle_bad_witness_rejected(gpu_ctx):
    """A wrong Merkle root in the public inputs and a corrupted RAM read are both caught."""
    import zkl_hip
    n = 1 << 9
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0601, 9, 6)
    opts = zkl_hip.proof_options(w, n, queries=8, grind=0)
    pi.merkle_root[3] ^= 0x10
    with pytest.raises(zkl_hip.ZklError, match="degree too large"):
        gpu_ctx.prove_segment(t, w, n, pi, opts)
    pi.merkle_root[3] ^= 0x10
    s_on, s_val, s_w = 149, 152, 153
    row = next(r for r in range(n) if t[s_on * n + r].lo == 1 and t[s_w * n + r].lo == 0
               and (t[s_val * n + r].lo | t[s_val * n + r].hi))
    t[s_val * n + row].lo ^= 1
    with pytest.raises(zkl_hip.ZklError, match="degree too large"):
        gpu_ctx.prove_segment(t, w, n, pi, opts)


def test_ram_full_size_verifies(oracle, gpu_ctx):
    """configs[1] shape (2^16 rows, blowup 16, q 64, grind 16) with sponge + RAM + Merkle."""
    import zkl_hip
    n = 1 << 16
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0700, 16, 7)
    assert w == 219
    opts = zkl_hip.proof_options(w, n)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    _, opi, _ = oracle.synth_segment(0x5EED0700, 16, 7)
    rc, err = oracle.verify(got, opi, oo)
    assert rc == 0, err


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


def test_full_size_deterministic_and_verifies(oracle, gpu_ctx):
    """BASELINE config: 65536 rows, blowup 16, q 64, grind 16; two runs give the same bytes
    and the proof passes the oracle verifier (OOD identity, all Merkle openings, DEEP,
    every FRI fold, remainder, proof of work)."""
    import zkl_hip
    n = 1 << 16
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0001, 16)
    opts = zkl_hip.proof_options(w, n)
    assert (opts.num_partitions, opts.hash_rate) == (4, 16)
    a = gpu_ctx.prove_segment(t, w, n, pi, opts)
    b = gpu_ctx.prove_segment(t, w, n, pi, opts)
    assert a == b
    print("full-size proof", len(a), hashlib.sha256(a).hexdigest(), gpu_ctx.stage_times())
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    _, opi, _ = oracle.synth_segment(0x5EED0001, 16)
    rc, err = oracle.verify(a, opi, oo)
    assert rc == 0, err
    bad = bytearray(a)
    bad[len(a) // 2] ^= 4
    assert oracle.verify(bytes(bad), opi, oo)[0] != 0


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


def test_stage_merkle_every_level_form(oracle, gpu_ctx):
    """A 2^17-leaf tree walks every level form launch_merkle picks (poseidon.hip:571-589): the
    32-state matrix-core levels (2^16, 2^15 nodes), the 16-state ones (2^14, 2^13), a lane-group
    level (2^12) and the 48-lane tree tops (<= 2^11, three launches); every node is compared with
    the oracle's merge (hasher.rs merge), not only the root."""
    rng = random.Random(17)
    P = oracle.P
    n = 1 << 17
    leaves = [rng.randrange(P) for _ in range(n)]
    raw = (C.c_uint8 * (16 * n)).from_buffer_copy(b"".join(v.to_bytes(16, "little") for v in leaves))
    d_l = gpu_ctx.alloc(16 * n)
    d_nodes = gpu_ctx.alloc(2 * n * 16)
    gpu_ctx.upload(d_l, raw, len(raw))
    gpu_ctx.merkle_tree(d_l, n, d_nodes)
    nodes = gpu_ctx.download(d_nodes, 2 * n * 16)
    got = [int.from_bytes(nodes[16 * i:16 * i + 16], "little") for i in range(2 * n)]
    assert got[n:] == leaves
    lvl, base = leaves, n
    while base > 1:
        lvl = [oracle.merge(lvl[2 * i], lvl[2 * i + 1]) for i in range(len(lvl) // 2)]
        base //= 2
        bad = [i for i in range(base) if got[base + i] != lvl[i]]
        assert not bad, f"level of {base} nodes: {len(bad)} nodes differ, first {bad[:4]}"
    for d in (d_l, d_nodes):
        gpu_ctx.free(d)


@pytest.mark.parametrize("log_n,blow", [(6, 16), (6, 8), (6, 2), (5, 32), (9, 4)])
def test_stage_lde_matches_oracle(oracle, gpu_ctx, log_n, blow):
    """zkl_hip_lde: coefficients and coset LDE (GENERATOR * <w_{blow*n}>) vs direct evaluation."""
    rng = random.Random(9)
    P = oracle.P
    ncols, n = 3, 1 << log_n
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
    g = oracle.root_of_unity(log_n)
    w = oracle.root_of_unity(log_n + blow.bit_length() - 1)
    for c in range(ncols):
        cs = [int.from_bytes(coef[16 * (c * n + k):16 * (c * n + k + 1)], "little") for k in range(n)]
        for r in (0, 5, n - 1):
            x = pow(g, r, P)
            assert sum(cs[k] * pow(x, k, P) for k in range(n)) % P == vals[c * n + r]
        for i in (0, 1, 17, N - 1):
            x = 3 * pow(w, i, P) % P
            want = sum(cs[k] * pow(x, k, P) for k in range(n)) % P
            assert int.from_bytes(lde[16 * (c * N + i):16 * (c * N + i + 1)], "little") == want
    for d in (d_v, d_c, d_l):
        gpu_ctx.free(d)


@pytest.mark.parametrize("log_n", [1, 3, 8, 9, 10, 12])
def test_stage_ntt_dif_dit(oracle, gpu_ctx, log_n):
    """zkl_hip_ntt: DIF (natural -> bit-reversed) and DIT (bit-reversed -> natural), forward
    and inverse, against direct evaluation at sampled outputs; sizes below and at the
    context's twiddle-table size (log_n 12 forces a table rebuild)."""
    rng = random.Random(11 + log_n)
    P = oracle.P
    n, ncols = 1 << log_n, 2
    w = oracle.root_of_unity(log_n)
    wi = pow(w, P - 2, P)
    vals = [rng.randrange(P) for _ in range(ncols * n)]
    raw = (C.c_uint8 * (16 * ncols * n)).from_buffer_copy(b"".join(v.to_bytes(16, "little") for v in vals))
    d = gpu_ctx.alloc(len(raw))

    def br(k):
        return int(format(k, f"0{log_n}b")[::-1], 2) if log_n else 0

    def get(buf, c, i):
        return int.from_bytes(buf[16 * (c * n + i):16 * (c * n + i + 1)], "little")

    samples = sorted({0, 1, n // 2, n - 1, rng.randrange(n), rng.randrange(n)})
    for inverse in (False, True):
        root = wi if inverse else w
        # DIF: natural in, out[bitrev(k)] = sum_j a_j root^(jk)
        gpu_ctx.upload(d, raw, len(raw))
        gpu_ctx.ntt(d, ncols, n, dif=True, inverse=inverse)
        out = gpu_ctx.download(d, len(raw))
        for c in range(ncols):
            a = vals[c * n:(c + 1) * n]
            for k in samples:
                want = sum(a[j] * pow(root, j * k, P) for j in range(n)) % P
                assert get(out, c, br(k)) == want, (inverse, c, k)
        # DIT: bit-reversed in, natural out: feed a[bitrev(j)] at position j
        perm = [vals[c * n + br(j)] for c in range(ncols) for j in range(n)]
        praw = (C.c_uint8 * (16 * ncols * n)).from_buffer_copy(b"".join(v.to_bytes(16, "little") for v in perm))
        gpu_ctx.upload(d, praw, len(praw))
        gpu_ctx.ntt(d, ncols, n, dif=False, inverse=inverse)
        out = gpu_ctx.download(d, len(raw))
        for c in range(ncols):
            a = vals[c * n:(c + 1) * n]
            for k in samples:
                want = sum(a[j] * pow(root, j * k, P) for j in range(n)) % P
                assert get(out, c, k) == want, ("dit", inverse, c, k)
    gpu_ctx.free(d)


def test_concurrent_contexts_same_device(gpu_ctx):
    """Several contexts proving different segments at once on one device (threads; the
    ctypes calls release the GIL) give the same bytes as one context proving them in turn:
    per-proof constants are per context, not module-global."""
    import threading
    import zkl_hip
    n = 1 << 9
    jobs = []
    for k in range(3):
        t, pi, w = zkl_hip.synth_vm_segment(0x5EED0200 + k, 9)
        opts = zkl_hip.proof_options(w, n, queries=16, grind=4)
        jobs.append((t, pi, w, opts))
    want = [gpu_ctx.prove_segment(t, w, n, pi, o) for t, pi, w, o in jobs]
    ctxs = [zkl_hip.Context(0) for _ in jobs]
    got = [None] * len(jobs)

    def run(i):
        t, pi, w, o = jobs[i]
        for _ in range(3):
            got[i] = ctxs[i].prove_segment(t, w, n, pi, o)

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(jobs))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for c in ctxs:
        c.close()
    assert got == want


@pytest.mark.parametrize("change,msg", [
    (dict(log_n=4), "power of two >= 32"),
    (dict(blowup=4), "blowup factor below"),
    (dict(blowup=12), "power of two"),
    (dict(queries=0), "num_queries"),
    (dict(field_extension=2), "FieldExtension::None"),
    (dict(width_delta=1), "width"),
])
def test_invalid_requests_rejected(gpu_ctx, change, msg):
    """Unsupported or inconsistent requests fail with ZKL_E_INVALID and a message, never a
    proof (the reference maps such failures to prove::Error, prove.rs:225-227)."""
    import zkl_hip
    log_n = change.get("log_n", 6)
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0300, max(log_n, 5))
    n = 1 << log_n
    opts = zkl_hip.proof_options(w, 1 << max(log_n, 5), queries=change.get("queries", 8),
                                 blowup=change.get("blowup", 16), grind=0)
    if "field_extension" in change:
        opts.field_extension = change["field_extension"]
    w_req = w - change.get("width_delta", 0)
    with pytest.raises(zkl_hip.ZklError, match=msg):
        gpu_ctx.prove_segment(t, w_req, n, pi, opts)


@pytest.mark.slow
def test_c5_shape_2p20_rows_verifies(oracle, gpu_ctx):
    """BASELINE configs[4] shape: one 2^20-row segment (LDE 2^24 x 204 = 55 GB in HBM,
    partitions (16,16) -> 13 row partitions).  The oracle prover is too slow at this size,
    so the proof is checked by the oracle verifier (plus a one-byte corruption)."""
    import zkl_hip
    oracle.set_threads(16)
    n = 1 << 20
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0020, 20)
    opts = zkl_hip.proof_options(w, n)
    assert (opts.num_partitions, opts.hash_rate) == (16, 16)
    proof = gpu_ctx.prove_segment(t, w, n, pi, opts)
    print("2^20 proof", len(proof), gpu_ctx.stage_times())
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    _, opi, _ = oracle.synth_segment(0x5EED0020, 20)
    rc, err = oracle.verify(proof, opi, oo)
    oracle.set_threads(1)
    assert rc == 0, err


@pytest.fixture
def pm_policy(gpu_ctx):
    """Route every Poseidon level of >= 32 states to the matrix-core permutation, restore the
    default policy afterwards."""
    import zkl_hip
    lib = zkl_hip.load_library()
    assert lib.zkl_hip_set_hash_policy(1, 32) == 0
    yield
    assert lib.zkl_hip_set_hash_policy(1, 1 << 14) == 0


def _fe_buf(vals):
    return (C.c_uint8 * (16 * len(vals))).from_buffer_copy(b"".join(v.to_bytes(16, "little") for v in vals))


@pytest.mark.parametrize("engine", [1, 0, 2])
def test_stage_permute_matches_oracle(oracle, gpu_ctx, engine):
    """zkl_hip_poseidon_permute (the 32- and 16-state matrix-core forms, the lane-group form) vs the oracle permutation, on
    random states, a partial last batch and the extreme elements 0, 1, p-1, 2^127."""
    rng = random.Random(11 + engine)
    P = oracle.P
    n = 1000
    edge = [0, 1, P - 1, 1 << 127, P - 2, (1 << 64) - 1, 1 << 64]
    states = [[e] * 12 for e in edge] + [[rng.choice(edge) for _ in range(12)] for _ in range(9)]
    states += [[rng.randrange(P) for _ in range(12)] for _ in range(n - len(states))]
    flat = [x for s in states for x in s]
    d = gpu_ctx.alloc(16 * len(flat))
    gpu_ctx.upload(d, _fe_buf(flat), 16 * len(flat))
    gpu_ctx.poseidon_permute(d, n, engine)
    got = gpu_ctx.download(d, 16 * len(flat))
    gpu_ctx.free(d)
    for i in list(range(40)) + list(range(40, n, 37)) + [n - 1]:
        want = oracle.permute(states[i])
        have = [int.from_bytes(got[16 * (12 * i + j):16 * (12 * i + j) + 16], "little") for j in range(12)]
        assert have == want, f"state {i}"


def _row_digest(oracle, row, np_, rate=16):
    ncols = len(row)
    psize = ncols
    if np_ > 1:
        psize = max(-(-ncols // np_), rate)
    if psize == ncols:
        return oracle.hash_elements(row)
    return oracle.merge_many([oracle.hash_elements(row[c:c + psize]) for c in range(0, ncols, psize)])


@pytest.mark.parametrize("ncols,nrows,np_", [
    (51, 1000, 1),     # one partition, partial last batch of 32 rows
    (204, 1056, 4),    # trace commitment shape (4 x 51 + merge_many)
    (256, 544, 16),    # 16 partitions: merge_many absorbs over two blocks
    (180, 96, 9),      # 9 partitions: the last count whose digests stay in registers
    (160, 64, 10),     # 10 partitions: the LDS digest buffer form
    (7, 2048, 4),      # composition shape (one 16-wide partition + merge_many)
    (33, 96, 2),
])
def test_stage_hash_rows_matrix_core(oracle, gpu_ctx, pm_policy, ncols, nrows, np_):
    rng = random.Random(ncols * 7 + nrows)
    P = oracle.P
    vals = [rng.randrange(P) for _ in range(ncols * nrows)]
    raw = _fe_buf(vals)
    d_m = gpu_ctx.alloc(len(raw))
    d_o = gpu_ctx.alloc(nrows * 16)
    d_nodes = gpu_ctx.alloc(2 * 1024 * 16)
    gpu_ctx.upload(d_m, raw, len(raw))
    gpu_ctx.hash_rows(d_m, ncols, nrows, np_, 16, d_o)
    got = gpu_ctx.download(d_o, nrows * 16)
    for r in sorted(set(list(range(0, nrows, 53)) + [nrows - 1, 31, 32])):
        row = [vals[c * nrows + r] for c in range(ncols)]
        assert int.from_bytes(got[16 * r:16 * r + 16], "little") == _row_digest(oracle, row, np_), f"row {r}"
    if nrows >= 1024:  # Merkle tree over the first 1024 digests (levels of 512..32 on the matrix cores)
        gpu_ctx.merkle_tree(d_o, 1024, d_nodes)
        nodes = gpu_ctx.download(d_nodes, 2 * 1024 * 16)
        lvl = [int.from_bytes(got[16 * i:16 * i + 16], "little") for i in range(1024)]
        while len(lvl) > 1:
            lvl = [oracle.merge(lvl[2 * i], lvl[2 * i + 1]) for i in range(len(lvl) // 2)]
        assert int.from_bytes(nodes[16:32], "little") == lvl[0]
    for d in (d_m, d_o, d_nodes):
        gpu_ctx.free(d)


@pytest.mark.parametrize("log_n,q,blowup,grind,flags", [
    (6, 32, 16, 4, 0), (8, 64, 16, 8, 0), (7, 40, 8, 2, 1), (6, 16, 16, 2, 2),
])
def test_proof_bytes_match_oracle_matrix_core(oracle, gpu_ctx, pm_policy, log_n, q, blowup, grind, flags):
    """Every commitment level of >= 32 states (trace/composition rows, Merkle levels, FRI
    leaves) on the matrix-core permutation: proof bytes still equal the oracle's."""
    import zkl_hip
    n = 1 << log_n
    seed = 0x3C0DE00 + log_n + 16 * flags
    t, pi, w = zkl_hip.synth_vm_segment(seed, log_n, flags)
    opts = zkl_hip.proof_options(w, n, queries=q, blowup=blowup, grind=grind)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    ot, opi, _ = oracle.synth_segment(seed, log_n, flags)
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    want = oracle.prove(ot, w, n, opi, oo)
    assert got == want


def test_step_proof_of_gpu_proof(oracle, gpu_ctx):
    """zl1 step proof (a18) around a GPU inner proof: the ZKLSTP1 bytes, root_trace and step
    digest equal the oracle's around the oracle's proof of the same segment."""
    import zkl_hip
    n = 1 << 7
    t, pi, w = zkl_hip.synth_vm_segment(0x57E9A007, 7)
    opts = zkl_hip.proof_options(w, n, queries=16, grind=4)
    inner = gpu_ctx.prove_segment(t, w, n, pi, opts)
    info = zkl_hip.StepInfo()
    info.suite_id[:] = bytes(pi.program_id)
    info.lambda_bits, info.segment_index, info.segments_total = 96, 3, 8
    info.state_in_hash[:] = bytes(range(32))
    step = zkl_hip.step_proof_encode(pi, info, inner)
    ot, opi, _ = oracle.synth_segment(0x57E9A007, 7)
    oo = oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
    want = oracle.step_encode(opi, info, oracle.prove(ot, w, n, opi, oo))
    assert step == want
    assert zkl_hip.step_proof_digest(step) == oracle.step_digest(want)


@pytest.mark.parametrize("ncols,log_n,blow", [(64, 10, 8), (204, 9, 16), (3, 12, 2), (7, 6, 64)])
def test_lde_lazy_ntt_matches_canonical(gpu_ctx, ncols, log_n, blow):
    """The lazily reduced DIT passes (default) give the same LDE bytes as the canonical-form
    kernel, on inputs biased towards p - 1 (largest limbs) and random elements."""
    import zkl_hip
    lib = zkl_hip.load_library()
    rng = random.Random(ncols + log_n)
    P = 2**128 - 45 * 2**40 + 1
    n = 1 << log_n
    N = n * blow
    vals = [P - 1 - rng.randrange(2**20) if rng.random() < 0.5 else rng.randrange(P) for _ in range(ncols * n)]
    raw = (C.c_uint8 * (16 * ncols * n)).from_buffer_copy(b"".join(v.to_bytes(16, "little") for v in vals))
    d_v, d_c, d_l = gpu_ctx.alloc(len(raw)), gpu_ctx.alloc(len(raw)), gpu_ctx.alloc(16 * ncols * N)
    gpu_ctx.upload(d_v, raw, len(raw))
    outs = []
    try:
        for lazy in (0, 1):
            assert lib.zkl_hip_set_ntt_mode(lazy) == 0
            gpu_ctx.lde(d_v, ncols, n, blow, d_c, d_l)
            outs.append(gpu_ctx.download(d_l, 16 * ncols * N))
    finally:
        lib.zkl_hip_set_ntt_mode(1)
        for d in (d_v, d_c, d_l):
            gpu_ctx.free(d)
    assert outs[0] == outs[1]


def test_full_size_proof_independent_of_kernel_forms(gpu_ctx):
    """configs[1] shape (2^16 rows, blowup 16, q 64, grind 16): the proof bytes are the same
    with the matrix-core or the lane-group permutation on every level and with the lazy or
    the canonical DIT NTT — each form is checked against the others at full size."""
    import zkl_hip
    lib = zkl_hip.load_library()
    n = 1 << 16
    t, pi, w = zkl_hip.synth_vm_segment(0x5EEDF00D, 16)
    opts = zkl_hip.proof_options(w, n)
    proofs = {}
    try:
        for name, engine, min_items, lazy in (("default", 1, 1 << 14, 1), ("lane", 0, 1 << 14, 1),
                                              ("all_mfma", 1, 32, 1), ("canonical_ntt", 1, 1 << 14, 0)):
            assert lib.zkl_hip_set_hash_policy(engine, min_items) == 0
            assert lib.zkl_hip_set_ntt_mode(lazy) == 0
            proofs[name] = gpu_ctx.prove_segment(t, w, n, pi, opts)
    finally:
        lib.zkl_hip_set_hash_policy(1, 1 << 14)
        lib.zkl_hip_set_ntt_mode(1)
    ref = proofs["default"]
    assert all(p == ref for p in proofs.values()), [k for k, p in proofs.items() if p != ref]


# ---------------------------------------------------------------------------------------
# Headline configuration (BASELINE configs[1]: 2^16 rows, blowup 16, q 64, grind 16,
# partitions (4, 16)): proof bytes against the CPU oracle's, via the committed goldens
# (tests/golden/make_proof_goldens.py) and one direct oracle proof.  These cover the
# 4-partition trace row digest (4 x 51 columns + merge_many) and the one-chunk composition
# row digest (7 columns < partition size 16) at proof level.
# ---------------------------------------------------------------------------------------
def _goldens():
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "proof_2p16.json")
    return json.load(open(p))


@pytest.mark.parametrize("name", sorted(_goldens()))
def test_headline_proof_matches_golden(gpu_ctx, name):
    import zkl_hip
    g = _goldens()[name]
    n = 1 << g["log_n"]
    t, pi, w = zkl_hip.synth_vm_segment(g["seed"], g["log_n"], g["flags"])
    assert w == g["width"]
    opts = zkl_hip.proof_options(w, n)
    assert {f: getattr(opts, f) for f, _ in opts._fields_} == g["options"]
    assert (opts.num_partitions, opts.hash_rate) == (4, 16)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    assert len(got) == g["len"]
    assert hashlib.sha256(got).hexdigest() == g["sha256"]
    zkl_hip.verify_segment(got, pi, opts)  # product-side verifier (zkl_verify_segment)


def test_headline_proof_equals_oracle_proof(oracle, gpu_ctx):
    """One direct comparison at the headline configuration (no golden in between): the oracle
    proves the same 2^16-row segment on the host (~40 s on 16 threads)."""
    import os
    import zkl_hip
    n = 1 << 16
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0001, 16)
    opts = zkl_hip.proof_options(w, n)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    oracle.set_threads(int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    ot, opi, _ = oracle.synth_segment(0x5EED0001, 16)
    want = oracle.prove(ot, w, n, opi, _gpu_opts(oracle, opts))
    oracle.set_threads(1)
    assert got == want


def test_c3_pipeline_bytes_match_sequential_and_goldens(gpu_ctx):
    """configs[2] shape: 8 distinct 2^16-row segments proved by 4 contexts in flight on one
    device (the bench's in-GPU pipeline) give, per segment, the same bytes as one context
    proving them in turn, and those equal the oracle goldens."""
    import threading
    import zkl_hip
    gold = {g["seed"]: g for g in _goldens().values() if g["flags"] == 0}
    n = 1 << 16
    segs = []
    for i in range(8):
        t, pi, w = zkl_hip.synth_vm_segment(0x5EED0001 + i, 16)
        segs.append((t, pi, w, zkl_hip.proof_options(w, n)))
    seq = [gpu_ctx.prove_segment(t, w, n, pi, o) for t, pi, w, o in segs]
    ctxs = [zkl_hip.Context(0) for _ in range(4)]
    dev = []
    for k, (t, pi, w, o) in enumerate(segs):
        c = ctxs[k % 4]
        d = c.alloc(w * n * 16)
        c.upload(d, t, w * n * 16)
        dev.append(d)
    got = [None] * 8

    def run(k):
        for i in range(k, 8, 4):
            t, pi, w, o = segs[i]
            got[i] = ctxs[k].prove_segment_device(dev[i], w, n, pi, o)

    try:
        th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        for k, d in enumerate(dev):
            ctxs[k % 4].free(d)
        for c in ctxs:
            c.close()
    assert got == seq
    for i, p in enumerate(seq):
        g = gold[0x5EED0001 + i]
        assert len(p) == g["len"] and hashlib.sha256(p).hexdigest() == g["sha256"], f"segment {i}"


@pytest.mark.parametrize("rule", [0, 1])
def test_row_digest_rule_proofs_match_oracle(oracle, gpu_ctx, rule):
    """Both one-chunk row-digest rules on the GPU equal the oracle under the
    same rule, on a segment with partitions (2, 16): the trace rows form two chunks, the
    composition rows one (the rows the rules disagree on)."""
    import zkl_hip
    n = 1 << 8
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0A08, 8)
    opts = zkl_hip.proof_options(w, n, queries=24, grind=4)
    opts.num_partitions = 2
    with zkl_hip.row_digest_rule(rule):
        got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    ot, opi, _ = oracle.synth_segment(0x5EED0A08, 8)
    oracle.set_row_digest_rule(rule)
    try:
        want = oracle.prove(ot, w, n, opi, _gpu_opts(oracle, opts))
        assert oracle.verify(got, opi, _gpu_opts(oracle, opts))[0] == 0
    finally:
        oracle.set_row_digest_rule(0)
    assert got == want


@pytest.mark.parametrize("field,value,msg", [
    ("num_partitions", 17, "num_partitions"), ("num_partitions", 0, "num_partitions"),
    ("hash_rate", 300, "hash_rate"), ("fri_remainder_max_degree", 2, "fri_remainder_max_degree"),
])
def test_invalid_partition_options_rejected(gpu_ctx, field, value, msg):
    import zkl_hip
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0300, 6)
    opts = zkl_hip.proof_options(w, 64, queries=8, grind=0)
    setattr(opts, field, value)
    with pytest.raises(zkl_hip.ZklError, match=msg):
        gpu_ctx.prove_segment(t, w, 64, pi, opts)


def _chain():
    import json
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "chain_2p16.json")
    return json.load(open(p)) if os.path.exists(p) else None


def _prove_chain(K, inflight=4):
    """The first K segments of the synthetic chained program, proved on the GPU by `inflight`
    contexts (one host thread each, the reference's bounded segment pool prove.rs:1018-1050),
    wrapped as zl1 steps of a K-segment program.  Returns (proofs, steps, public inputs)."""
    import threading
    import zkl_hip
    ch = _chain()
    n = 1 << ch["log_n"]
    ctxs = [zkl_hip.Context(0) for _ in range(inflight)]
    dev, pis, got = [], [], [None] * K
    try:
        for k in range(K):  # one host trace at a time: 64 x 214 MB stays in HBM only
            t, pi, w = zkl_hip.synth_vm_segment_chain(ch["program_seed"], ch["program_seed"] + k, ch["log_n"],
                                                      int(ch["rom0_in"][k], 16))
            d = ctxs[k % inflight].alloc(w * n * 16)
            ctxs[k % inflight].upload(d, t, w * n * 16)
            dev.append((d, w))
            pis.append(pi)
            del t

        def run(k):
            for i in range(k, K, inflight):
                d, w = dev[i]
                got[i] = ctxs[k].prove_segment_device(d, w, n, pis[i], zkl_hip.proof_options(w, n))

        th = [threading.Thread(target=run, args=(k,)) for k in range(inflight)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        for k, (d, _) in enumerate(dev):
            ctxs[k % inflight].free(d)
        for c in ctxs:
            c.close()
    steps = []
    for i, (pi, p) in enumerate(zip(pis, got)):
        info = zkl_hip.step_info_for(pi, i, K, i.to_bytes(32, "little"), (i + 1).to_bytes(32, "little"))
        steps.append(zkl_hip.step_proof_encode(pi, info, p))
    return got, steps, pis


def _check_segments(got):
    ch = _chain()
    for i, p in enumerate(got):
        g = ch["segments"][i]
        assert g["index"] == i and len(p) == g["len"] and hashlib.sha256(p).hexdigest() == g["sha256"], f"segment {i}"


@pytest.mark.skipif(_chain() is None, reason="tests/golden/chain_2p16.json not generated")
def test_chain_program_and_aggregation_match_goldens(oracle, gpu_ctx):
    """BASELINE configs[2] end to end: the first 8 segments of the synthetic multi-segment
    program (tests/golden/make_chain_goldens.py), proved on the GPU with 4 contexts in flight,
    equal the oracle goldens; their zl1 steps aggregate (zkl_agg_prove, FieldExtension::
    Quadratic) into the golden ZKLRC1 artifact and recursion digest, and into the artifact
    oracle/agg_ref.py builds from the GPU steps."""
    import sys
    import zkl_hip
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import agg_ref
    ch = _chain()
    got, steps, _ = _prove_chain(8)
    _check_segments(got)
    art, dg = zkl_hip.agg_prove(steps)
    ga = ch["aggregation"]
    assert ga["children"] == 8
    assert len(art) == ga["len"] and hashlib.sha256(art).hexdigest() == ga["sha256"]
    assert dg.hex() == ga["recursion_digest"]
    want, want_dg, _ = agg_ref.agg_prove(oracle, steps)
    assert art == want and dg == want_dg
    zkl_hip.agg_verify(art)


@pytest.mark.skipif(_chain() is None or "aggregation_64" not in _chain() or len(_chain()["segments"]) < 64,
                    reason="64-segment chain goldens not generated")
def test_chain_64_segments_and_aggregation_match_goldens(gpu_ctx):
    """BASELINE configs[3] on one GPU: all 64 segments of the chained program (prove.rs:1018-
    1050), 4 contexts in flight, equal the 64 oracle goldens; the 64 zl1 steps aggregate
    (lib.rs:295-551) into the golden 64-child ZKLRC1 artifact (oracle/agg_ref.py over the
    oracle's step proofs) and recursion digest, and the product verifier accepts it.  The
    8-GPU run shards exactly these segments (bench.py --gpus 8, zkl_hip/dist.py).

    The reference-trace aggregation mode (agg/trace.rs:397-398 row count, hash_row_poseidon
    root errors 553-600) at real size: the first 16 segments as a 16-step program give the
    golden `aggregation_ref_trace` artifact (16-row trace, like the published run's), and all 64
    give `aggregation_64_ref_trace` (64 rows: no padding row).  With ZKL_DUMP_CHAIN=<dir> the
    proof bytes are written there (make_chain_goldens.py --from-dir uses them)."""
    import zkl_hip
    ch = _chain()
    got, steps, pis = _prove_chain(64)
    _check_segments(got)
    dump = os.environ.get("ZKL_DUMP_CHAIN")
    if dump:
        os.makedirs(dump, exist_ok=True)
        for i, p in enumerate(got):
            open(os.path.join(dump, f"seg{i:02d}.bin"), "wb").write(p)
    art, dg = zkl_hip.agg_prove(steps)
    ga = ch["aggregation_64"]
    assert ga["children"] == 64
    assert len(art) == ga["len"] and hashlib.sha256(art).hexdigest() == ga["sha256"]
    assert dg.hex() == ga["recursion_digest"]
    zkl_hip.agg_verify(art)
    T = zkl_hip.agg_trace(steps)
    assert len(T[0]) == 128  # next_pow2(max(64 + 1, 8)): the padding row
    ref16 = []
    for i in range(16):  # the first 16 proofs as steps of a 16-segment program
        pi = pis[i]
        info = zkl_hip.step_info_for(pi, i, 16, i.to_bytes(32, "little"), (i + 1).to_bytes(32, "little"))
        ref16.append(zkl_hip.step_proof_encode(pi, info, got[i]))
    for key, st, rows in (("aggregation_ref_trace", ref16, 16), ("aggregation_64_ref_trace", steps, 64)):
        g = ch.get(key)
        if g is None:
            continue
        art, dg = zkl_hip.agg_prove(st, trace_mode=zkl_hip.AGG_TRACE_REFERENCE)
        assert g["children"] == len(st)
        assert (len(art), hashlib.sha256(art).hexdigest(), dg.hex()) == (g["len"], g["sha256"], g["recursion_digest"]), key
        assert len(zkl_hip.agg_trace(st, trace_mode=zkl_hip.AGG_TRACE_REFERENCE)[0]) == rows


@pytest.mark.parametrize("log_n,width_flags", [(16, 0), (18, 0), (12, 2)])
def test_host_trace_chunked_upload_matches_device_entry(gpu_ctx, log_n, width_flags):
    """zkl_hip_prove_segment with a pageable host trace (column chunks through the pinned ring,
    each chunk's LDE issued as its DMA lands) gives the proof zkl_hip_prove_segment_device gives
    for the same trace resident in HBM: chunk sizes of 16 / 4 / 256 columns, widths 204 and 212
    (the last chunk partial)."""
    import zkl_hip
    n = 1 << log_n
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0B00 + log_n, log_n, width_flags)
    opts = zkl_hip.proof_options(w, n, queries=16, grind=4)
    host = gpu_ctx.prove_segment(t, w, n, pi, opts)
    assert gpu_ctx.host_times()["upload"] > 0
    d = gpu_ctx.alloc(w * n * 16)
    try:
        gpu_ctx.upload(d, t, w * n * 16)
        dev = gpu_ctx.prove_segment_device(d, w, n, pi, opts)
    finally:
        gpu_ctx.free(d)
    assert host == dev
    zkl_hip.verify_segment(host, pi, opts)


def test_prove_into_caller_buffer(gpu_ctx):
    """zkl_hip_prove_segment_device_into writes the same bytes zkl_hip_prove_segment_device
    returns; a buffer one byte short fails with the size named and zkl_hip_last_proof still
    returns the proof; after a failed prove call no proof is held."""
    import zkl_hip
    log_n = 12
    n = 1 << log_n
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED1700, log_n, 0)
    opts = zkl_hip.proof_options(w, n, queries=16, grind=4)
    d = gpu_ctx.alloc(w * n * 16)
    try:
        gpu_ctx.upload(d, t, w * n * 16)
        ref = gpu_ctx.prove_segment_device(d, w, n, pi, opts)
        assert gpu_ctx.last_proof() == ref
        buf = bytearray(len(ref) + 100)
        ln = gpu_ctx.prove_segment_device_into(d, w, n, pi, opts, buf)
        assert ln == len(ref) and bytes(buf[:ln]) == ref
        short = bytearray(len(ref) - 1)
        with pytest.raises(zkl_hip.ZklError, match=f"{len(ref)} bytes needed"):
            gpu_ctx.prove_segment_device_into(d, w, n, pi, opts, short)
        assert gpu_ctx.last_proof() == ref
        bad = zkl_hip.proof_options(w, n, queries=16, grind=4)
        bad.blowup_factor = 3  # not a power of two: rejected before any device work
        with pytest.raises(zkl_hip.ZklError):
            gpu_ctx.prove_segment_device_into(d, w, n, pi, bad, buf)
        with pytest.raises(zkl_hip.ZklError, match="no proof"):
            gpu_ctx.last_proof()
    finally:
        gpu_ctx.free(d)


@pytest.mark.parametrize("flags,blowup", [(0, 8), (0, 16), (0, 32), (0, 64), (1, 16), (2, 8)])
def test_split_lde_layout_proofs_match_oracle(oracle, gpu_ctx, flags, blowup):
    """2^8-row segments are the smallest whose trace LDE ends in an 8-stage register pass, so
    the prover stores it in the split layout: blowup 8 puts every LDE row in the
    CE domain (the evaluator reads all positions), 16 the even rows (first half only), 32 and 64
    every 4th / 8th row (the evaluator walks CE points and looks rows up); sponge (flags 1) and
    RAM/Merkle (flags 2) layouts add their AIR blocks.  Proof bytes equal the oracle's (natural
    order throughout)."""
    import zkl_hip
    oracle.set_threads(1)
    n = 1 << 8
    seed = 0x5E1170 + 16 * flags + blowup
    t, pi, w = zkl_hip.synth_vm_segment(seed, 8, flags)
    opts = zkl_hip.proof_options(w, n, queries=32, blowup=blowup, grind=4)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    ot, opi, _ = oracle.synth_segment(seed, 8, flags)
    want = oracle.prove(ot, w, n, opi, oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_]))
    assert got == want


def test_remainder_degree_boundary_prove_then_verify(oracle, gpu_ctx):
    """the largest remainder degree the verifier accepts at a blowup (7 at blowup 8)
    proves, equals the oracle's proof and verifies with the product verifier; one step further
    (15) is refused by the prover as by the verifier."""
    import zkl_hip
    log_n = 8
    n = 1 << log_n
    trace, pi, w = zkl_hip.synth_vm_segment(0x5EED0B08, log_n)
    opts = zkl_hip.proof_options(w, n, queries=16, blowup=8, grind=4)
    opts.fri_remainder_max_degree = 7
    got = gpu_ctx.prove_segment(trace, w, n, pi, opts)
    ot, opi, _ = oracle.synth_segment(0x5EED0B08, log_n)
    want = oracle.prove(ot, w, n, opi, oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_]))
    assert got == want
    zkl_hip.verify_segment(got, pi, opts)
    opts.fri_remainder_max_degree = 15
    with pytest.raises(zkl_hip.ZklError, match="below the blowup factor"):
        gpu_ctx.prove_segment(trace, w, n, pi, opts)

