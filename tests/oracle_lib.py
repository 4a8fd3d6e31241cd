"""ctypes bindings to the C oracle (oracle/liboracle_zkl.so).

ORACLE = test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg load this.  The product (libzkl_hip.so) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle_zkl.so")

P = 2**128 - 45 * 2**40 + 1

_lib = None


class F128(C.Structure):
    _fields_ = [("lo", C.c_uint64), ("hi", C.c_uint64)]


class ProofOptions(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "num_queries", "blowup_factor", "grinding_factor", "field_extension",
        "fri_folding_factor", "fri_remainder_max_degree", "batching_constraints",
        "batching_deep", "num_partitions", "hash_rate")]


class AirPublicInputs(C.Structure):
    _fields_ = [
        ("program_id", C.c_uint8 * 32),
        ("program_commitment", C.c_uint8 * 32),
        ("merkle_root", C.c_uint8 * 32),
        ("feature_mask", C.c_uint64),
        ("segment_feature_mask", C.c_uint64),
        ("n_main_slots", C.c_uint32),
        ("main_slots", F128 * 8),
        ("vm_out_reg", C.c_uint32),
        ("vm_out_row", C.c_uint32),
        ("vm_expected_bytes", C.c_uint8 * 32),
        ("rom_acc", F128 * 3),
        ("pc_init", F128),
        ("ram_gp_unsorted_in", F128),
        ("ram_gp_unsorted_out", F128),
        ("ram_gp_sorted_in", F128),
        ("ram_gp_sorted_out", F128),
        ("rom_s_in", F128 * 3),
        ("rom_s_out", F128 * 3),
        ("vm_usage_mask", C.c_uint32),
        ("ram_delta_clk_bits", C.c_uint32),
    ]


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_prove_segment.restype = C.c_int
        _lib.orc_last_error.restype = C.c_char_p
        _lib.orc_api_air_info.restype = C.c_int
    return _lib


def fe_bytes(x):
    return (x % P).to_bytes(16, "little")


def fe_from(b):
    return int.from_bytes(bytes(b), "little")


def _buf(n):
    return (C.c_uint8 * n)()


def fe_mul(a, b):
    o = _buf(16)
    lib().orc_api_fe_mul(fe_bytes(a), fe_bytes(b), o)
    return fe_from(o)


def fe_add(a, b):
    o = _buf(16)
    lib().orc_api_fe_add(fe_bytes(a), fe_bytes(b), o)
    return fe_from(o)


def fe_sub(a, b):
    o = _buf(16)
    lib().orc_api_fe_sub(fe_bytes(a), fe_bytes(b), o)
    return fe_from(o)


def fe_inv(a):
    o = _buf(16)
    lib().orc_api_fe_inv(fe_bytes(a), o)
    return fe_from(o)


def root_of_unity(k):
    o = _buf(16)
    lib().orc_api_root_of_unity(C.c_uint(k), o)
    return fe_from(o)


def blake3(data: bytes) -> bytes:
    o = _buf(32)
    lib().orc_blake3(data, C.c_size_t(len(data)), o)
    return bytes(o)


def suite(sid: bytes, rounds=27):
    dom, mds, rc = _buf(32), _buf(144 * 16), _buf(rounds * 12 * 16)
    lib().orc_api_suite(sid, C.c_int(rounds), dom, mds, rc)
    d = bytes(dom)
    m = bytes(mds)
    r = bytes(rc)
    return ([fe_from(d[0:16]), fe_from(d[16:32])],
            [[fe_from(m[16 * (12 * i + j):16 * (12 * i + j + 1)]) for j in range(12)] for i in range(12)],
            [[fe_from(r[16 * (12 * k + j):16 * (12 * k + j + 1)]) for j in range(12)] for k in range(rounds)])


def permute(state):
    src = b"".join(fe_bytes(x) for x in state)
    o = _buf(12 * 16)
    lib().orc_api_permute(src, o)
    ob = bytes(o)
    return [fe_from(ob[16 * i:16 * i + 16]) for i in range(12)]


def hash_elements(elems):
    o = _buf(16)
    lib().orc_api_hash_elements(b"".join(fe_bytes(x) for x in elems), C.c_size_t(len(elems)), o)
    return fe_from(o)


def merge(a, b):
    o = _buf(16)
    lib().orc_api_merge(fe_bytes(a), fe_bytes(b), o)
    return fe_from(o)


def merge_many(ds):
    o = _buf(16)
    lib().orc_api_merge_many(b"".join(fe_bytes(x) for x in ds), C.c_size_t(len(ds)), o)
    return fe_from(o)


def merge_with_int(s, v):
    o = _buf(16)
    lib().orc_api_merge_with_int(fe_bytes(s), C.c_uint64(v), o)
    return fe_from(o)


def hash_bytes(data: bytes):
    o = _buf(16)
    lib().orc_api_hash_bytes(data, C.c_size_t(len(data)), o)
    return fe_from(o)


def program_field_commitment(b32: bytes):
    o = _buf(32)
    lib().orc_api_program_field_commitment(b32, o)
    ob = bytes(o)
    return fe_from(ob[:16]), fe_from(ob[16:])


def synth_segment(seed: int, log_n: int, flags: int = 0):
    """Returns (trace as (F128 * (W*n)) column-major, AirPublicInputs, W).
    flags bit 0: program with sponge ops (features VM | SPONGE | POSEIDON)."""
    w = C.c_uint32()
    lib().orc_synth_vm_segment_ex(C.c_uint64(seed), C.c_uint32(log_n), C.c_uint32(flags), None, None, C.byref(w))
    n = 1 << log_n
    trace = (F128 * (w.value * n))()
    pi = AirPublicInputs()
    rc = lib().orc_synth_vm_segment_ex(C.c_uint64(seed), C.c_uint32(log_n), C.c_uint32(flags), trace, C.byref(pi),
                                       C.byref(w))
    assert rc == 0
    return trace, pi, w.value


def synth_segment_chain(program_seed: int, seed: int, log_n: int, rom0: int = 0, flags: int = 0):
    """orc_synth_vm_segment_chain: segment `seed` of program `program_seed`, ROM lane 0
    entering at rom0.  Returns (trace, AirPublicInputs, W)."""
    w = C.c_uint32()
    r0 = F128(rom0 & (2 ** 64 - 1), rom0 >> 64)
    lib().orc_synth_vm_segment_chain(C.c_uint64(program_seed), C.c_uint64(seed), C.c_uint32(log_n),
                                     C.c_uint32(flags), C.byref(r0), None, None, C.byref(w))
    n = 1 << log_n
    trace = (F128 * (w.value * n))()
    pi = AirPublicInputs()
    rc = lib().orc_synth_vm_segment_chain(C.c_uint64(program_seed), C.c_uint64(seed), C.c_uint32(log_n),
                                          C.c_uint32(flags), C.byref(r0), trace, C.byref(pi), C.byref(w))
    assert rc == 0
    return trace, pi, w.value


def build_trace(ops, program_id: bytes, program_commitment: bytes | None = None, secret_args=(), main_args=None,
                rom0: int = 0):
    """orc_build_trace over a ctypes array of zkl_op (the product's zkl_hip.ZklOp layout) and
    VmArg main args (ctypes array or None).  Returns (rc, trace, AirPublicInputs, W, n_rows)."""
    commit = bytes(program_commitment if program_commitment is not None else program_id)
    sec = (C.c_uint64 * max(1, len(secret_args)))(*secret_args)
    n_main = 0 if main_args is None else len(main_args)
    ma = None if main_args is None else C.cast(main_args, C.c_void_p)
    r0 = F128(rom0 & (2 ** 64 - 1), rom0 >> 64)
    w, n = C.c_uint32(), C.c_uint32()
    args = (C.cast(ops, C.c_void_p), C.c_uint32(len(ops)), bytes(program_id), commit, sec, C.c_uint32(len(secret_args)),
            ma, C.c_uint32(n_main), C.byref(r0))
    rc = lib().orc_build_trace(*args, None, None, C.byref(w), C.byref(n))
    if rc != 0:
        return rc, None, None, 0, 0
    trace = (F128 * (w.value * n.value))()
    pi = AirPublicInputs()
    rc = lib().orc_build_trace(*args, trace, C.byref(pi), C.byref(w), C.byref(n))
    return rc, trace, pi, w.value, n.value


def build_segment_trace(ops, program_id: bytes, r_start: int, r_end: int, program_commitment: bytes | None = None,
                        secret_args=(), main_args=None, rom0: int = 0):
    """orc_build_segment_trace (zkl_build_segment_trace's twin: every level streamed, no full
    trace).  Returns (rc, trace, AirPublicInputs, W, state_in, state_out)."""
    commit = bytes(program_commitment if program_commitment is not None else program_id)
    sec = (C.c_uint64 * max(1, len(secret_args)))(*secret_args)
    n_main = 0 if main_args is None else len(main_args)
    ma = None if main_args is None else C.cast(main_args, C.c_void_p)
    r0 = F128(rom0 & (2 ** 64 - 1), rom0 >> 64)
    w = C.c_uint32()
    args = (C.cast(ops, C.c_void_p), C.c_uint32(len(ops)), bytes(program_id), commit, sec, C.c_uint32(len(secret_args)),
            ma, C.c_uint32(n_main), C.byref(r0), C.c_uint32(r_start), C.c_uint32(r_end))
    rc = lib().orc_build_segment_trace(*args, None, None, C.byref(w), None, None)
    if rc != 0:
        return rc, None, None, 0, None, None
    trace = (F128 * (w.value * (r_end - r_start)))()
    pi = AirPublicInputs()
    sin, sout = (C.c_uint8 * 32)(), (C.c_uint8 * 32)()
    rc = lib().orc_build_segment_trace(*args, trace, C.byref(pi), C.byref(w), sin, sout)
    return rc, trace, pi, w.value, bytes(sin), bytes(sout)


def default_options(width, n, queries=64, blowup=16, grind=16):
    parts = 16 if n >= 1 << 20 else 8 if n >= 1 << 18 else 4 if n >= 1 << 16 else 2 if n >= 1 << 14 else 1
    rate = 8 if width <= 32 else 16
    return ProofOptions(queries, blowup, grind, 1, 2, 1, 0, 0, parts, rate)


def air_info(pi, width, n):
    ntc, na, ceb, nc = C.c_int(), C.c_size_t(), C.c_int(), C.c_int()
    rc = lib().orc_api_air_info(C.byref(pi), C.c_uint32(width), C.c_size_t(n), C.byref(ntc),
                                C.byref(na), C.byref(ceb), C.byref(nc))
    return rc, ntc.value, na.value, ceb.value, nc.value


def check_trace(trace, pi, width, n):
    br, bi = C.c_size_t(), C.c_int()
    rc = lib().orc_api_check_trace(trace, C.c_uint32(width), C.c_size_t(n), C.byref(pi), C.byref(br), C.byref(bi))
    return rc, br.value, bi.value


def set_row_digest_rule(rule):
    """0: winterfell commit_to_rows (default); 1: agg/child.rs:1025-1045 hash_row_poseidon."""
    lib().orc_set_row_digest_rule(C.c_int(rule))


def row_digest_rule():
    return lib().orc_row_digest_rule()


def row_digest(row, psize):
    o = _buf(16)
    lib().orc_api_row_digest(b"".join(fe_bytes(x) for x in row), C.c_size_t(len(row)), C.c_size_t(psize), o)
    return fe_from(o)


def partition_size(np_, rate, ncols):
    """PartitionOptions::partition_size for the base field (ExtensionDegree 1)."""
    return ncols if np_ <= 1 else max(-(-ncols // np_), rate)


def set_threads(t):
    lib().orc_set_threads(C.c_int(t))


def prove(trace, width, n, pi, opts, boundary_mode=0):
    out = C.POINTER(C.c_uint8)()
    ln = C.c_size_t()
    rc = lib().orc_prove_segment(trace, C.c_uint32(width), C.c_uint32(n), C.byref(pi), C.byref(opts),
                                 C.byref(out), C.byref(ln), C.c_int(boundary_mode))
    if rc != 0:
        raise RuntimeError(f"oracle prove failed rc={rc}: {lib().orc_last_error().decode()}")
    data = bytes(out[:ln.value])
    lib().orc_free(out)
    return data


def verify(proof: bytes, pi, opts):
    err = C.create_string_buffer(256)
    rc = lib().orc_verify_segment(proof, C.c_size_t(len(proof)), C.byref(pi), C.byref(opts), err, C.c_size_t(256))
    return rc, err.value.decode()


def last_times():
    arr = (C.c_double * 8)()
    lib().orc_last_times(arr)
    return list(arr)


def step_encode(pi, info, inner: bytes) -> bytes:
    """oracle/step.c: StepProof::to_bytes restatement (info: zkl_hip.StepInfo layout)."""
    out = C.POINTER(C.c_uint8)()
    ln = C.c_size_t()
    rc = lib().orc_step_encode(C.byref(pi), C.byref(info), inner, C.c_size_t(len(inner)), C.byref(out), C.byref(ln))
    if rc != 0:
        raise ValueError("oracle step encode failed")
    data = bytes(out[:ln.value])
    lib().orc_free(out)
    return data


def children_root(suite: bytes, digests, roots) -> bytes:
    """oracle/step.c: agg::child::children_root_from_compact restatement."""
    out = (C.c_uint8 * 32)()
    lib().orc_children_root(bytes(suite), b"".join(digests), b"".join(roots), C.c_uint32(len(digests)), out)
    return bytes(out)


def step_digest(step: bytes):
    """oracle/step.c: (digest, root_trace) or raises ValueError(message)."""
    d, r = (C.c_uint8 * 32)(), (C.c_uint8 * 32)()
    err = C.create_string_buffer(256)
    rc = lib().orc_step_digest(step, C.c_size_t(len(step)), d, r, err, C.c_size_t(256))
    if rc != 0:
        raise ValueError(err.value.decode())
    return bytes(d), bytes(r)
