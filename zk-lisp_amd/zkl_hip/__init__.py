"""zkl_hip — Python host for the MI355X-native zk-lisp segment prover.

Mirrors the reference's prove path for one execution segment:
  ZkProver::prove (zk-lisp-proof-winterfell/src/prove.rs:174-257)
    -> winterfell::Prover::prove with ZkLispAir + PoseidonHasher (prove.rs:425-517)
through the C ABI of libzkl_hip.so (include/zkl_hip.h).  The shared library is built
in-tree by zk-lisp_amd/Makefile; importing this module fails loudly when it is missing.
There is no CPU fallback: every proof is produced by the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import os

__all__ = [
    "F128", "ProofOptions", "AirPublicInputs", "ZklError", "Context", "load_library",
    "select_partitions_for_trace", "proof_options", "synth_vm_segment", "STAGE_NAMES",
    "FM_VM", "FM_VM_EXPECT", "FM_POSEIDON", "FM_SPONGE", "FM_MERKLE", "FM_RAM",
    "VmArg", "StepInfo", "check_request", "row_digest_rule", "verify_segment", "step_proof_encode", "step_proof_digest", "parse_step_proof", "children_root",
    "AggOptions", "agg_prove", "agg_verify", "agg_trace", "parse_agg_artifact", "synth_segment_chain", "synth_vm_segment_chain",
    "step_info_for", "ZklOp", "op", "build_trace", "OP_KINDS", "rom_acc_from_program", "plan_segments", "slice_segment",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libzkl_hip.so")

# feature bits, zk-lisp-proof/src/pi.rs:23-28
FM_POSEIDON, FM_VM, FM_VM_EXPECT, FM_SPONGE, FM_MERKLE, FM_RAM = 1, 2, 16, 32, 64, 128

STAGE_NAMES = ["trace_lde", "trace_commit", "evaluator", "constraint_commitment", "ood",
               "deep", "fri", "grind", "queries", "finish"]

ERRORS = {-1: "invalid", -2: "device", -3: "oom", -4: "internal"}


class ZklError(RuntimeError):
    """Mirrors prove::Error::Backend(String) (prove.rs:52-62)."""

    def __init__(self, code, msg):
        super().__init__(f"backend error ({ERRORS.get(code, code)}): {msg}")
        self.code = code


class F128(C.Structure):
    _fields_ = [("lo", C.c_uint64), ("hi", C.c_uint64)]


class ProofOptions(C.Structure):
    """winterfell::ProofOptions as built at prove.rs:963-972 (+ with_partitions, :1121)."""
    _fields_ = [(n, C.c_uint32) for n in (
        "num_queries", "blowup_factor", "grinding_factor", "field_extension",
        "fri_folding_factor", "fri_remainder_max_degree", "batching_constraints",
        "batching_deep", "num_partitions", "hash_rate")]


class AirPublicInputs(C.Structure):
    """crate::AirPublicInputs (lib.rs:75-95) with the PublicInputs subset the AIR reads."""
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


class VmArg(C.Structure):
    """zk_lisp_proof::pi::VmArg: tag 0 = U64, 1 = U128 (LE bytes), 2 = Bytes32."""
    _fields_ = [("tag", C.c_uint32), ("bytes", C.c_uint8 * 32)]


class StepInfo(C.Structure):
    """zkl_step_info: what prove_segment (prove.rs:1057-1175) passes to the zl1 wrapper
    besides the inner proof and the AirPublicInputs."""
    _fields_ = [
        ("suite_id", C.c_uint8 * 32),
        ("lambda_bits", C.c_uint32),
        ("segment_index", C.c_uint32),
        ("segments_total", C.c_uint32),
        ("pc_init", C.c_uint8 * 32),
        ("state_in_hash", C.c_uint8 * 32),
        ("state_out_hash", C.c_uint8 * 32),
        ("ram_gp_unsorted_in", C.c_uint8 * 32),
        ("ram_gp_unsorted_out", C.c_uint8 * 32),
        ("ram_gp_sorted_in", C.c_uint8 * 32),
        ("ram_gp_sorted_out", C.c_uint8 * 32),
        ("rom_s_in", (C.c_uint8 * 32) * 3),
        ("rom_s_out", (C.c_uint8 * 32) * 3),
        ("n_main_args", C.c_uint32),
        ("main_args", VmArg * 8),
    ]


_lib = None


def load_library():
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("ZKL_HIP_LIB", LIB_PATH)  # tools/: benchmark a variant build
    if not os.path.exists(path):
        raise ImportError(f"libzkl_hip.so not built ({path}); run `make -C zk-lisp_amd`")
    lib = C.CDLL(path)
    P = C.POINTER
    lib.zkl_hip_init.argtypes = [C.c_int, P(C.c_void_p)]
    lib.zkl_hip_destroy.argtypes = [C.c_void_p]
    lib.zkl_hip_last_error.argtypes = [C.c_void_p]
    lib.zkl_hip_last_error.restype = C.c_char_p
    lib.zkl_hip_free.argtypes = [C.c_void_p]
    lib.zkl_hip_prove_segment.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                          P(AirPublicInputs), P(ProofOptions), P(P(C.c_uint8)), P(C.c_size_t)]
    lib.zkl_hip_prove_segment_device.argtypes = lib.zkl_hip_prove_segment.argtypes
    lib.zkl_hip_prove_segment_device_into.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                                      P(AirPublicInputs), P(ProofOptions), C.c_void_p, C.c_size_t,
                                                      P(C.c_size_t)]
    lib.zkl_hip_last_proof.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, P(C.c_size_t)]
    lib.zkl_hip_stage_times.argtypes = [C.c_void_p, P(C.c_double), C.c_int]
    lib.zkl_hip_host_times.argtypes = [C.c_void_p, P(C.c_double), C.c_int]
    lib.zkl_hip_kernel_times.argtypes = [C.c_void_p, P(C.c_double), P(C.c_int), C.c_int, P(C.c_char_p)]
    lib.zkl_hip_device_count.argtypes = [P(C.c_int)]
    lib.zkl_hip_device_alloc.argtypes = [C.c_void_p, C.c_size_t, P(C.c_void_p)]
    lib.zkl_hip_device_free.argtypes = [C.c_void_p, C.c_void_p]
    lib.zkl_hip_memcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    lib.zkl_hip_synchronize.argtypes = [C.c_void_p]
    lib.zkl_select_partitions.argtypes = [C.c_uint32, C.c_uint32, P(C.c_uint32), P(C.c_uint32)]
    lib.zkl_synth_vm_segment.argtypes = [C.c_uint64, C.c_uint32, C.c_void_p, P(AirPublicInputs), P(C.c_uint32)]
    lib.zkl_synth_vm_segment_ex.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p, P(AirPublicInputs),
                                            P(C.c_uint32)]
    lib.zkl_hip_ntt.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int]
    lib.zkl_hip_hash_rows.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
    lib.zkl_hip_merkle_tree.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]
    lib.zkl_hip_poseidon_permute.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int]
    lib.zkl_hip_set_hash_policy.argtypes = [C.c_int, C.c_uint32]
    lib.zkl_hip_set_ntt_mode.argtypes = [C.c_int]
    lib.zkl_hip_set_row_digest_rule.argtypes = [C.c_int]
    lib.zkl_verify_segment.argtypes = [C.c_char_p, C.c_size_t, P(AirPublicInputs), P(ProofOptions)]
    lib.zkl_hip_check_request.argtypes = [C.c_uint32, C.c_uint32, P(AirPublicInputs), P(ProofOptions)]
    lib.zkl_hip_set_kernel_timing.argtypes = [C.c_void_p, C.c_int]
    lib.zkl_step_proof_encode.argtypes = [P(AirPublicInputs), P(StepInfo), C.c_char_p, C.c_size_t,
                                          P(P(C.c_uint8)), P(C.c_size_t)]
    lib.zkl_step_proof_digest.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_void_p]
    lib.zkl_children_root.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint32, C.c_void_p]
    lib.zkl_hip_lde.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]
    lib.zkl_synth_vm_segment_chain.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, P(F128), C.c_void_p,
                                               P(AirPublicInputs), P(C.c_uint32)]
    lib.zkl_build_trace.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                    C.c_uint32, P(F128), C.c_void_p, P(AirPublicInputs), P(C.c_uint32),
                                    P(C.c_uint32)]
    lib.zkl_rom_acc_from_program.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, P(F128)]
    lib.zkl_plan_segments.argtypes = [C.c_uint32, C.c_uint32, P(C.c_uint32), P(C.c_uint32), C.c_uint32, P(C.c_uint32)]
    lib.zkl_slice_segment.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, P(AirPublicInputs),
                                      C.c_uint32, C.c_uint32, C.c_void_p, P(AirPublicInputs), P(C.c_uint32),
                                      C.c_void_p, C.c_void_p]
    lib.zkl_hip_process_tuning.argtypes = [C.c_uint32, P(C.c_uint32)]
    lib.zkl_hip_trace_buffer.argtypes = [C.c_void_p, C.c_uint32, C.c_size_t, P(C.c_void_p)]
    if hasattr(lib, "zkl_hip_pinned_bytes"):  # (older builds, loaded by tools/ for A/B, lack it)
        lib.zkl_hip_pinned_bytes.argtypes = [P(C.c_uint64), P(C.c_uint64)]
    lib.zkl_program_new.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                    C.c_uint32, P(F128), P(C.c_void_p), P(C.c_uint32), P(C.c_uint32)]
    lib.zkl_build_segment_trace.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, P(AirPublicInputs),
                                            P(C.c_uint32), C.c_void_p, C.c_void_p]
    lib.zkl_program_free.argtypes = [C.c_void_p]
    lib.zkl_agg_prove.argtypes = [P(C.c_char_p), P(C.c_size_t), C.c_uint32, P(AggOptions), P(P(C.c_uint8)),
                                  P(C.c_size_t), C.c_void_p]
    lib.zkl_agg_verify.argtypes = [C.c_char_p, C.c_size_t, C.c_uint32]
    lib.zkl_agg_trace.argtypes = [P(C.c_char_p), P(C.c_size_t), C.c_uint32, C.c_void_p, C.c_uint32, P(C.c_uint32)]
    lib.zkl_agg_trace_mode.argtypes = [P(C.c_char_p), P(C.c_size_t), C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32,
                                       P(C.c_uint32)]
    lib.zkl_comm_unique_id.argtypes = [C.c_void_p]
    lib.zkl_comm_available.argtypes = []
    lib.zkl_comm_init.argtypes = [C.c_int, C.c_int, C.c_int, C.c_char_p, P(C.c_void_p)]
    lib.zkl_comm_gather_bytes.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_int, P(P(C.c_uint8)),
                                          P(C.c_size_t)]
    lib.zkl_comm_last_ms.argtypes = [C.c_void_p]
    lib.zkl_comm_last_ms.restype = C.c_double
    lib.zkl_comm_destroy.argtypes = [C.c_void_p]
    _lib = lib
    return lib


class AggOptions(C.Structure):
    """zk_lisp_proof::ProverOptions as the aggregation reads it (zk-lisp-proof/src/lib.rs:40-66)."""
    _fields_ = [("queries", C.c_uint32), ("blowup", C.c_uint32), ("grind", C.c_uint32),
                ("min_security_bits", C.c_uint32), ("trace_mode", C.c_uint32)]


AGG_TRACE_VALID = 0      # ZKL_AGG_TRACE_VALID: one padding row, zero root errors (proof.bin)
AGG_TRACE_REFERENCE = 1  # ZKL_AGG_TRACE_REFERENCE: agg/trace.rs's own trace bytes


def _steps_args(steps):
    arr = (C.c_char_p * len(steps))(*[bytes(s) for s in steps])
    lens = (C.c_size_t * len(steps))(*[len(s) for s in steps])
    return arr, lens


def agg_prove(steps, queries=64, blowup=16, grind=16, min_security_bits=128, trace_mode=AGG_TRACE_VALID):
    """RecursionPublicBuilder::build_public + RecursionBackend::prove + RecursionArtifactCodec::
    encode (lib.rs:295-551): ZKLSTP1 step proofs -> (ZKLRC1 artifact, recursion digest)."""
    lib = load_library()
    arr, lens = _steps_args(steps)
    o = AggOptions(queries, blowup, grind, min_security_bits, trace_mode)
    out, ln, dg = C.POINTER(C.c_uint8)(), C.c_size_t(), (C.c_uint8 * 32)()
    rc = lib.zkl_agg_prove(arr, lens, len(steps), C.byref(o), C.byref(out), C.byref(ln), dg)
    if rc:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode(errors="replace"))
    data = C.string_at(out, ln.value)
    lib.zkl_hip_free(out)
    return data, bytes(dg)


def agg_verify(artifact: bytes, min_security_bits: int = 128) -> None:
    """RecursionArtifactCodec::decode + RecursionBackend::verify (verify_agg_proof, prove.rs:732-791)
    of a ZKLRC1 artifact; raises ZklError naming the failing check."""
    lib = load_library()
    rc = lib.zkl_agg_verify(bytes(artifact), len(artifact), min_security_bits)
    if rc:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode(errors="replace"))


def agg_trace(steps, trace_mode=AGG_TRACE_VALID):
    """build_agg_trace_from_transcripts (agg/trace.rs:155-238): 31 column lists of ints."""
    lib = load_library()
    arr, lens = _steps_args(steps)
    rows = C.c_uint32()
    rc = lib.zkl_agg_trace_mode(arr, lens, len(steps), trace_mode, None, 0, C.byref(rows))
    if rc:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode(errors="replace"))
    buf = (F128 * (31 * rows.value))()
    rc = lib.zkl_agg_trace_mode(arr, lens, len(steps), trace_mode, C.cast(buf, C.c_void_p), rows.value,
                                C.byref(rows))
    if rc:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode(errors="replace"))
    r = rows.value
    return [[buf[c * r + i].lo | (buf[c * r + i].hi << 64) for i in range(r)] for c in range(31)]


def parse_agg_artifact(b: bytes) -> dict:
    """RecursionArtifactCodec::decode (lib.rs:552-...) field order: the ZKLRC1 public inputs and
    the aggregation proof bytes."""
    import struct
    if b[:6] != b"ZKLRC1":
        raise ValueError("invalid recursion artifact magic")
    off = 6

    def take(k):
        nonlocal off
        if off + k > len(b):
            raise ValueError("recursion artifact truncated")
        off += k
        return b[off - k:off]

    d = {k: take(32) for k in ("program_id", "program_commitment", "pi_digest", "children_root", "batch_id")}
    d["v_units_total"], d["children_count"] = struct.unpack("<QI", take(12))
    d["m"], d["rho"], d["q"], d["o"], d["lambda"], d["pi_len"], d["v_units"] = struct.unpack("<IHHHHIQ", take(24))
    d["lde_blowup"], d["folding_factor"], d["redundancy"], d["num_layers"] = struct.unpack("<IBBB", take(7))
    d["num_queries"], d["grinding_factor"] = struct.unpack("<HI", take(6))
    d["suite_id"] = take(32)
    n_ms = struct.unpack("<I", take(4))[0]
    d["children_ms"] = list(struct.unpack(f"<{n_ms}I", take(4 * n_ms)))
    for k in ("vm_state_initial", "vm_state_final", "ram_gp_unsorted_initial", "ram_gp_unsorted_final",
              "ram_gp_sorted_initial", "ram_gp_sorted_final"):
        d[k] = take(32)
    d["rom_s_initial"] = [take(32) for _ in range(3)]
    d["rom_s_final"] = [take(32) for _ in range(3)]
    d["proof"] = take(struct.unpack("<I", take(4))[0])
    if off != len(b):
        raise ValueError("trailing bytes after the recursion artifact")
    return d


def step_info_for(pi: AirPublicInputs, index: int, total: int, state_in: bytes, state_out: bytes,
                  lambda_bits: int = 128, main_args=()) -> "StepInfo":
    """zl1 step metadata as prove_segment fills it (prove.rs:1103-1174): suite = program_id
    (prove.rs:985), the segment boundary bytes fe_to_bytes_fold of the AIR public inputs'
    pc_init / RAM grand products / ROM lanes (SegmentBoundaryBytes, prove.rs:1112), the VM
    state hashes of the trace builder (here given) and the program's typed main args (the
    PublicInputs::main_args the zl1 proof carries; ints or (tag, bytes) as build_trace takes)."""
    info = StepInfo()
    if len(main_args) > 8:
        raise ValueError("at most 8 main args")
    info.n_main_args = len(main_args)
    va = _vm_args(list(main_args))
    for i in range(len(main_args)):
        info.main_args[i] = va[i]
    info.suite_id[:] = bytes(pi.program_id)
    info.lambda_bits, info.segment_index, info.segments_total = lambda_bits, index, total

    def fold(v):
        return (v.lo | (v.hi << 64)).to_bytes(16, "little") + bytes(16)

    info.pc_init[:] = fold(pi.pc_init)
    info.state_in_hash[:] = bytes(state_in)
    info.state_out_hash[:] = bytes(state_out)
    for f in ("ram_gp_unsorted_in", "ram_gp_unsorted_out", "ram_gp_sorted_in", "ram_gp_sorted_out"):
        getattr(info, f)[:] = fold(getattr(pi, f))
    for i in range(3):
        info.rom_s_in[i][:] = fold(pi.rom_s_in[i])
        info.rom_s_out[i][:] = fold(pi.rom_s_out[i])
    return info


def synth_vm_segment_chain(program_seed: int, seed: int, log_n: int, rom0: int = 0, flags: int = 0):
    """One segment of a synthetic multi-segment program (zkl_synth_vm_segment_chain): program
    identity from program_seed, ops from seed, ROM lane 0 entering at rom0.  (trace, pi, width)."""
    lib = load_library()
    w = C.c_uint32()
    r0 = F128(rom0 & (2 ** 64 - 1), rom0 >> 64)
    lib.zkl_synth_vm_segment_chain(program_seed, seed, log_n, flags, C.byref(r0), None, None, C.byref(w))
    trace = (F128 * (w.value * (1 << log_n)))()
    pi = AirPublicInputs()
    rc = lib.zkl_synth_vm_segment_chain(program_seed, seed, log_n, flags, C.byref(r0), C.cast(trace, C.c_void_p),
                                        C.byref(pi), C.byref(w))
    if rc != 0:
        raise ZklError(rc, "synth_vm_segment_chain failed")
    return trace, pi, w.value


def synth_segment_chain(seed: int, log_n: int, count: int, flags: int = 0):
    """`count` synthetic segments of one program (program id from `seed`, ops from seed + i) whose
    ROM accumulator lane 0 carries from one to the next (zkl_synth_vm_segment_chain):
    [(trace, pi, width)]; segment i+1 starts where segment i's
    rom_s_out[0] ended, as the aggregation's ROM chain requires (agg/trace.rs:524-541)."""
    lib = load_library()
    out, rom0 = [], F128(0, 0)
    for i in range(count):
        w = C.c_uint32()
        lib.zkl_synth_vm_segment_chain(seed, seed + i, log_n, flags, None, None, None, C.byref(w))
        trace = (F128 * (w.value * (1 << log_n)))()
        pi = AirPublicInputs()
        rc = lib.zkl_synth_vm_segment_chain(seed, seed + i, log_n, flags, C.byref(rom0), C.cast(trace, C.c_void_p),
                                            C.byref(pi), C.byref(w))
        if rc != 0:
            raise ZklError(rc, "synth_vm_segment_chain failed")
        out.append((trace, pi, w.value))
        rom0 = F128(pi.rom_s_out[0].lo, pi.rom_s_out[0].hi)
    return out


def check_request(width: int, n_rows: int, pi: AirPublicInputs, opts: ProofOptions) -> None:
    """The prover's request checks without a device (zkl_hip_check_request); raises ZklError
    with the prover's message, as prove_segment would before any device work."""
    lib = load_library()
    rc = lib.zkl_hip_check_request(width, n_rows, C.byref(pi), C.byref(opts))
    if rc != 0:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode(errors="replace"))


def verify_segment(proof: bytes, pi: AirPublicInputs, opts: ProofOptions) -> None:
    """winter-verifier checks of one segment proof on the host (zkl_verify_segment; the
    reference's verify_proof, prove.rs:802-941).  Raises ZklError naming the failing check."""
    lib = load_library()
    rc = lib.zkl_verify_segment(bytes(proof), len(proof), C.byref(pi), C.byref(opts))
    if rc != 0:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode(errors="replace"))


class row_digest_rule:
    """Context manager selecting the one-chunk row-digest rule (zkl_hip_set_row_digest_rule):
    0 winterfell commit_to_rows (default), 1 agg/child.rs:1025-1045 hash_row_poseidon."""

    def __init__(self, rule: int):
        self.rule = rule

    def __enter__(self):
        lib = load_library()
        self.prev = lib.zkl_hip_row_digest_rule()
        if lib.zkl_hip_set_row_digest_rule(self.rule) != 0:
            raise ZklError(-1, f"invalid row digest rule {self.rule}")
        return self

    def __exit__(self, *exc):
        load_library().zkl_hip_set_row_digest_rule(self.prev)
        return False


def device_count() -> int:
    lib = load_library()
    n = C.c_int()
    rc = lib.zkl_hip_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def select_partitions_for_trace(width: int, length: int):
    """utils::select_partitions_for_trace (utils.rs:394-409)."""
    lib = load_library()
    np_, rate = C.c_uint32(), C.c_uint32()
    lib.zkl_select_partitions(width, length, C.byref(np_), C.byref(rate))
    return np_.value, rate.value


def step_proof_encode(pi: AirPublicInputs, info: StepInfo, inner: bytes) -> bytes:
    """StepProof::to_bytes (proof/step.rs:79-151) of the zl1 step proof around `inner`."""
    lib = load_library()
    out = C.POINTER(C.c_uint8)()
    ln = C.c_size_t()
    rc = lib.zkl_step_proof_encode(C.byref(pi), C.byref(info), inner, len(inner), C.byref(out), C.byref(ln))
    if rc:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode())
    data = C.string_at(out, ln.value)
    lib.zkl_hip_free(out)
    return data


def parse_step_proof(b: bytes) -> dict:
    """Host mirror of StepProof::from_bytes (proof/step.rs:153-493): the fields of a ZKLSTP1
    encoding, with the inner Winterfell proof bytes under "inner"."""
    import struct
    if len(b) < 7 or b[:7] != b"ZKLSTP1":
        raise ValueError("invalid step proof magic tag")
    off = 7

    def take(k, what):
        nonlocal off
        if off + k > len(b):
            raise ValueError(f"step proof truncated before {what}")
        off += k
        return b[off - k:off]

    d = {"lambda_bits": struct.unpack("<I", take(4, "lambda_bits"))[0], "suite_id": take(32, "suite_id"),
         "program_id": take(32, "program_id"), "program_commitment": take(32, "program_commitment"),
         "merkle_root": take(32, "merkle_root"), "feature_mask": struct.unpack("<Q", take(8, "feature_mask"))[0]}
    args = []
    for _ in range(struct.unpack("<I", take(4, "main_args length"))[0]):
        tag = take(1, "VmArg tag")[0]
        if tag > 2:
            raise ValueError("invalid VmArg tag in step proof encoding")
        args.append((tag, take({0: 8, 1: 16, 2: 32}[tag], "VmArg")))
    d["main_args"] = args
    d["vm_usage_mask"] = struct.unpack("<I", take(4, "vm_usage_mask"))[0]
    d["ram_delta_clk_bits"] = struct.unpack("<I", take(4, "ram_delta_clk_bits"))[0]
    d["rom_acc"] = [take(32, "rom_acc") for _ in range(3)]
    d["segment_index"] = struct.unpack("<I", take(4, "segment_index"))[0]
    d["segments_total"] = struct.unpack("<I", take(4, "segments_total"))[0]
    for f in ("pc_init", "state_in_hash", "state_out_hash", "ram_gp_unsorted_in", "ram_gp_unsorted_out",
              "ram_gp_sorted_in", "ram_gp_sorted_out"):
        d[f] = take(32, f)
    d["rom_s_in"] = [take(32, "rom_s_in") for _ in range(3)]
    d["rom_s_out"] = [take(32, "rom_s_out") for _ in range(3)]
    d["inner"] = take(struct.unpack("<I", take(4, "inner proof length"))[0], "inner proof bytes")
    if d["segments_total"] <= 1:  # new_single_segment (step.rs:413-432)
        d["segment_index"], d["segments_total"] = 0, 1
    return d


def children_root(suite_id: bytes, digests, root_traces) -> bytes:
    """agg::child::children_root_from_compact (agg/child.rs:853-895) over (step digest,
    zl1 root_trace) pairs of the children."""
    lib = load_library()
    out = (C.c_uint8 * 32)()
    digests, root_traces = [bytes(d) for d in digests], [bytes(r) for r in root_traces]
    if len(digests) != len(root_traces) or any(len(x) != 32 for x in digests + root_traces):
        raise ValueError("children_root: one 32-byte digest and one 32-byte root_trace per child")
    rc = lib.zkl_children_root(_id32("suite_id", suite_id), b"".join(digests), b"".join(root_traces), len(digests), out)
    if rc:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode())
    return bytes(out)


def step_proof_digest(step: bytes):
    """(step digest, zl1 root_trace) of a ZKLSTP1 encoding (digest.rs:16-68, format.rs:214-238)."""
    lib = load_library()
    d, r = (C.c_uint8 * 32)(), (C.c_uint8 * 32)()
    rc = lib.zkl_step_proof_digest(step, len(step), d, r)
    if rc:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode())
    return bytes(d), bytes(r)


def proof_options(width, length, queries=64, blowup=16, grind=16) -> ProofOptions:
    """ProofOptions::new(q, blowup, grind, None, 2, 1, Linear, Linear).with_partitions(...)."""
    parts, rate = select_partitions_for_trace(width, length)
    return ProofOptions(queries, blowup, grind, 1, 2, 1, 0, 0, parts, rate)


def synth_vm_segment(seed: int, log_n: int, flags: int = 0):
    """Synthetic VM segment (workload generator): returns (trace, pi, width), trace column-major.
    flags bit 0 adds sponge ops (FM_SPONGE | FM_POSEIDON segments)."""
    lib = load_library()
    w = C.c_uint32()
    lib.zkl_synth_vm_segment_ex(seed, log_n, flags, None, None, C.byref(w))
    n = 1 << log_n
    trace = (F128 * (w.value * n))()
    pi = AirPublicInputs()
    rc = lib.zkl_synth_vm_segment_ex(seed, log_n, flags, C.cast(trace, C.c_void_p), C.byref(pi), C.byref(w))
    if rc != 0:
        raise ZklError(rc, "synth_vm_segment failed")
    return trace, pi, w.value


def comm_available():
    """None when RCCL can be opened in this process, else the reason."""
    lib = load_library()
    return None if lib.zkl_comm_available() == 0 else lib.zkl_hip_last_error(None).decode(errors="replace")


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (zkl_comm_unique_id): 128 bytes the root hands to the other ranks."""
    lib = load_library()
    buf = (C.c_uint8 * 128)()
    rc = lib.zkl_comm_unique_id(buf)
    if rc:
        raise ZklError(rc, lib.zkl_hip_last_error(None).decode(errors="replace"))
    return bytes(buf)


class Comm:
    """RCCL communicator of one rank (zkl_comm_*): the multi-GPU boundary exchange of step
    proofs to the aggregating rank."""

    def __init__(self, device: int, world: int, rank: int, uid: bytes):
        self.lib = load_library()
        self.ptr = C.c_void_p()
        self.world, self.rank = world, rank
        rc = self.lib.zkl_comm_init(device, world, rank, bytes(uid), C.byref(self.ptr))
        if rc:
            raise ZklError(rc, self.lib.zkl_hip_last_error(None).decode(errors="replace"))

    def gather_bytes(self, data: bytes, root: int = 0):
        """Collective: list of every rank's bytes (rank order) on root, None elsewhere."""
        out = C.POINTER(C.c_uint8)()
        lens = (C.c_size_t * self.world)()
        rc = self.lib.zkl_comm_gather_bytes(self.ptr, bytes(data), len(data), root, C.byref(out), lens)
        if rc:
            raise ZklError(rc, self.lib.zkl_hip_last_error(None).decode(errors="replace"))
        if self.rank != root:
            return None
        blob = C.string_at(out, sum(lens)) if sum(lens) else b""
        self.lib.zkl_hip_free(out)
        res, off = [], 0
        for n in lens:
            res.append(blob[off:off + n])
            off += n
        return res

    def last_ms(self) -> float:
        return float(self.lib.zkl_comm_last_ms(self.ptr))

    def close(self):
        if self.ptr:
            self.lib.zkl_comm_destroy(self.ptr)
            self.ptr = C.c_void_p()


TUNE_SPIN, TUNE_MALLOC = 1, 2


def process_tuning(spin: bool = False, malloc: bool = False) -> dict:
    """zkl_hip_process_tuning: the opt-in process-wide settings (include/zkl_hip.h; zkl_hip_init
    changes nothing outside the library).  spin must come before the first Context of the
    process.  Returns {"spin": bool, "malloc": bool} of what took effect."""
    lib = load_library()
    flags = (TUNE_SPIN if spin else 0) | (TUNE_MALLOC if malloc else 0)
    got = C.c_uint32()
    lib.zkl_hip_process_tuning(flags, C.byref(got))
    return {"spin": bool(got.value & TUNE_SPIN), "malloc": bool(got.value & TUNE_MALLOC)}


class Context:
    """One prover context per device (zkl_hip_init)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        self.ptr = C.c_void_p()
        rc = self.lib.zkl_hip_init(device, C.byref(self.ptr))
        if rc != 0:
            raise ZklError(rc, self.lib.zkl_hip_last_error(None).decode())

    def close(self):
        if self.ptr:
            self.lib.zkl_hip_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, rc):
        raise ZklError(rc, self.lib.zkl_hip_last_error(self.ptr).decode())

    def _finish(self, rc, out, ln):
        if rc != 0:
            self._err(rc)
        data = C.string_at(out, ln.value)
        self.lib.zkl_hip_free(out)
        return data

    def prove_segment(self, trace, width: int, n_rows: int, pi: AirPublicInputs, opts: ProofOptions) -> bytes:
        """Proof::to_bytes() for one segment; `trace` is a host buffer (column-major f128)."""
        out = C.POINTER(C.c_uint8)()
        ln = C.c_size_t()
        ptr = trace if isinstance(trace, int) else C.cast(trace, C.c_void_p)
        rc = self.lib.zkl_hip_prove_segment(self.ptr, ptr, width, n_rows, C.byref(pi), C.byref(opts),
                                            C.byref(out), C.byref(ln))
        return self._finish(rc, out, ln)

    def trace_buffer(self, nbytes: int, slot: int = 0) -> int:
        """zkl_hip_trace_buffer: address of the context's pinned host trace buffer `slot` (0/1,
        >= nbytes), to be filled in place and passed to prove_segment (DMA'd without a staging
        copy)."""
        p = C.c_void_p()
        rc = self.lib.zkl_hip_trace_buffer(self.ptr, slot, nbytes, C.byref(p))
        if rc:
            self._err(rc)
        return p.value

    def prove_segment_device(self, d_trace_ptr: int, width: int, n_rows: int, pi, opts) -> bytes:
        """Same with the trace already resident in HBM (device pointer, e.g. torch data_ptr())."""
        out = C.POINTER(C.c_uint8)()
        ln = C.c_size_t()
        rc = self.lib.zkl_hip_prove_segment_device(self.ptr, C.c_void_p(d_trace_ptr), width, n_rows, C.byref(pi),
                                                   C.byref(opts), C.byref(out), C.byref(ln))
        return self._finish(rc, out, ln)

    def prove_segment_device_into(self, d_trace_ptr: int, width: int, n_rows: int, pi, opts, buf) -> int:
        """Same, written into `buf` (a writable ctypes / bytearray buffer kept across calls):
        returns the proof length; a buffer too small raises with the size in the message, and
        last_proof() still returns the bytes."""
        ln = C.c_size_t()
        cbuf = (C.c_uint8 * len(buf)).from_buffer(buf)
        rc = self.lib.zkl_hip_prove_segment_device_into(self.ptr, C.c_void_p(d_trace_ptr), width, n_rows, C.byref(pi),
                                                        C.byref(opts), cbuf, len(buf), C.byref(ln))
        if rc:
            self._err(rc)
        return ln.value

    def last_proof(self) -> bytes:
        """The last proof made on this context (valid until the next prove call)."""
        ln = C.c_size_t()
        rc = self.lib.zkl_hip_last_proof(self.ptr, None, 0, C.byref(ln))
        if rc:
            self._err(rc)
        buf = (C.c_uint8 * ln.value)()
        rc = self.lib.zkl_hip_last_proof(self.ptr, buf, ln.value, C.byref(ln))
        if rc:
            self._err(rc)
        return bytes(buf)

    def stage_times(self):
        arr = (C.c_double * len(STAGE_NAMES))()
        k = self.lib.zkl_hip_stage_times(self.ptr, arr, len(STAGE_NAMES))
        return dict(zip(STAGE_NAMES[:k], list(arr)[:k]))

    def host_times(self):
        """{setup, host_unoverlapped, call, upload} wall ms of the last proof (host side)."""
        arr = (C.c_double * 4)()
        k = self.lib.zkl_hip_host_times(self.ptr, arr, 4)
        return dict(zip(("setup", "host_unoverlapped", "call", "upload"), list(arr)[:k]))

    def kernel_times(self):
        """{family: (ms, launches)} of the last proof, from HIP events on the ctx stream."""
        ms = (C.c_double * 16)()
        cnt = (C.c_int * 16)()
        names = C.c_char_p()
        k = self.lib.zkl_hip_kernel_times(self.ptr, ms, cnt, 16, C.byref(names))
        fam = names.value.decode().split("\n")
        return {fam[i]: (ms[i], cnt[i]) for i in range(k)}

    # device memory owned by the library's HIP runtime
    def alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        rc = self.lib.zkl_hip_device_alloc(self.ptr, nbytes, C.byref(p))
        if rc:
            self._err(rc)
        return p.value

    def free(self, d_ptr: int):
        rc = self.lib.zkl_hip_device_free(self.ptr, C.c_void_p(d_ptr))
        if rc:
            self._err(rc)

    def upload(self, d_ptr: int, host_buf, nbytes: int):
        rc = self.lib.zkl_hip_memcpy(self.ptr, C.c_void_p(d_ptr), C.cast(host_buf, C.c_void_p), nbytes, 1)
        if rc:
            self._err(rc)

    def download(self, d_ptr: int, nbytes: int) -> bytes:
        buf = (C.c_uint8 * nbytes)()
        rc = self.lib.zkl_hip_memcpy(self.ptr, C.cast(buf, C.c_void_p), C.c_void_p(d_ptr), nbytes, 2)
        if rc:
            self._err(rc)
        return bytes(buf)

    def synchronize(self):
        rc = self.lib.zkl_hip_synchronize(self.ptr)
        if rc:
            self._err(rc)

    # stage entry points (device pointers)
    def hash_rows(self, d_mat, n_cols, n_rows, num_partitions, hash_rate, d_out):
        rc = self.lib.zkl_hip_hash_rows(self.ptr, C.c_void_p(d_mat), n_cols, n_rows, num_partitions, hash_rate,
                                        C.c_void_p(d_out))
        if rc:
            self._err(rc)

    def set_kernel_timing(self, mode: int):
        """0: no kernel-family events, 1: trace row hash only (default), 2: every family."""
        rc = self.lib.zkl_hip_set_kernel_timing(self.ptr, mode)
        if rc:
            self._err(rc)

    def poseidon_permute(self, d_states, n_states, engine=1):
        rc = self.lib.zkl_hip_poseidon_permute(self.ptr, C.c_void_p(d_states), n_states, engine)
        if rc:
            self._err(rc)

    def merkle_tree(self, d_leaves, n_leaves, d_nodes):
        rc = self.lib.zkl_hip_merkle_tree(self.ptr, C.c_void_p(d_leaves), n_leaves, C.c_void_p(d_nodes))
        if rc:
            self._err(rc)

    def ntt(self, d_data, n_cols, n, dif=True, inverse=False):
        rc = self.lib.zkl_hip_ntt(self.ptr, C.c_void_p(d_data), n_cols, n, int(dif), int(inverse))
        if rc:
            self._err(rc)

    def lde(self, d_values, n_cols, n_rows, blowup, d_coeffs, d_lde):
        rc = self.lib.zkl_hip_lde(self.ptr, C.c_void_p(d_values), n_cols, n_rows, blowup, C.c_void_p(d_coeffs),
                                  C.c_void_p(d_lde))
        if rc:
            self._err(rc)


class ZklOp(C.Structure):
    """zkl_op (include/zkl_hip.h): one zk_lisp_compiler::builder::Op (builder.rs:25-158)."""
    _fields_ = [("kind", C.c_uint32), ("dst", C.c_uint8), ("dst2", C.c_uint8), ("a", C.c_uint8), ("b", C.c_uint8),
                ("c", C.c_uint8), ("bits", C.c_uint8), ("n_regs", C.c_uint8), ("reserved", C.c_uint8),
                ("regs", C.c_uint8 * 10), ("imm", C.c_uint64)]


# builder::Op variant -> (ZKL_OP_* kind, {reference field name: zkl_op member})
OP_KINDS = {
    "Const": (0, {"dst": "dst", "imm": "imm"}),
    "Mov": (1, {"dst": "dst", "src": "a"}),
    "Add": (2, {"dst": "dst", "a": "a", "b": "b"}),
    "Sub": (3, {"dst": "dst", "a": "a", "b": "b"}),
    "Mul": (4, {"dst": "dst", "a": "a", "b": "b"}),
    "Neg": (5, {"dst": "dst", "a": "a"}),
    "Eq": (6, {"dst": "dst", "a": "a", "b": "b"}),
    "Select": (7, {"dst": "dst", "c": "c", "a": "a", "b": "b"}),
    "Assert": (8, {"dst": "dst", "c": "c"}),
    "AssertBit": (9, {"dst": "dst", "r": "c"}),
    "AssertRange": (10, {"dst": "dst", "r": "c", "bits": "bits"}),
    "AssertRangeLo": (11, {"dst": "dst", "r": "c"}),
    "AssertRangeHi": (12, {"dst": "dst", "r": "c"}),
    "DivMod": (13, {"dst_q": "dst", "dst_r": "dst2", "a": "a", "b": "b"}),
    "DivMod128": (14, {"a_hi": "a", "a_lo": "c", "b": "b", "dst_q": "dst", "dst_r": "dst2"}),
    "MulWide": (15, {"dst_hi": "dst2", "dst_lo": "dst", "a": "a", "b": "b"}),
    "Load": (16, {"dst": "dst", "addr": "a"}),
    "Store": (17, {"addr": "a", "src": "b"}),
    "SAbsorbN": (18, {"regs": "regs"}),
    "SSqueeze": (19, {"dst": "dst"}),
    "MerkleStepFirst": (20, {"leaf_reg": "dst", "dir_reg": "a", "sib_reg": "b"}),
    "MerkleStep": (21, {"dir_reg": "a", "sib_reg": "b"}),
    "MerkleStepLast": (22, {"dir_reg": "a", "sib_reg": "b"}),
    "End": (23, {}),
}


def op(name: str, **fields) -> ZklOp:
    """builder::Op by variant and field names, e.g. op("DivMod", dst_q=2, dst_r=3, a=0, b=1)."""
    if name not in OP_KINDS:
        raise ValueError(f"unknown op {name}")
    kind, members = OP_KINDS[name]
    if set(fields) != set(members):
        raise ValueError(f"{name} takes fields {sorted(members)}, got {sorted(fields)}")
    o = ZklOp()
    o.kind = kind
    for k, v in fields.items():
        m = members[k]
        if m == "regs":
            if not 1 <= len(v) <= 10:
                raise ValueError("SAbsorbN takes 1..10 registers")
            o.n_regs = len(v)
            o.regs[:len(v)] = list(v)
        else:
            setattr(o, m, v)
    return o


def _vm_args(main_args):
    """main_args as VmArg list: ints (< 2^64: U64, else U128) or (tag, bytes) pairs."""
    out = (VmArg * max(1, len(main_args)))()
    for i, a in enumerate(main_args):
        if isinstance(a, int):
            out[i].tag = 0 if a < 2 ** 64 else 1
            out[i].bytes[:16] = a.to_bytes(16, "little")
        else:
            out[i].tag = a[0]
            b = bytes(a[1])
            out[i].bytes[:len(b)] = b
    return out


def pinned_bytes():
    """(current, peak) bytes of pinned host memory the library holds (zkl_hip_pinned_bytes)."""
    lib = load_library()
    cur, peak = C.c_uint64(), C.c_uint64()
    if not hasattr(lib, "zkl_hip_pinned_bytes"):
        return 0, 0
    lib.zkl_hip_pinned_bytes(C.byref(cur), C.byref(peak))
    return cur.value, peak.value


def _id32(name: str, v) -> bytes:
    """A 32-byte program id / commitment argument: the C side reads exactly 32 bytes."""
    b = bytes(v)
    if len(b) != 32:
        raise ValueError(f"{name} must be 32 bytes, got {len(b)}")
    return b


def build_trace(ops, program_id: bytes, program_commitment: bytes | None = None, secret_args=(), main_args=(),
                rom0: int = 0):
    """build_full_trace (vm/trace/mod.rs:434-524) of an op list through zkl_build_trace:
    (trace, AirPublicInputs, width, n_rows), the trace column-major in the segment layout of the
    ops' features.  program_commitment defaults to program_id (the AIR binds pi_prog at row 0 to
    the commitment, air/mod.rs)."""
    lib = load_library()
    program_id = _id32("program_id", program_id)
    commit = _id32("program_commitment", program_commitment if program_commitment is not None else program_id)
    arr = (ZklOp * len(ops))(*ops)
    sec = (C.c_uint64 * max(1, len(secret_args)))(*secret_args)
    ma = _vm_args(list(main_args))
    r0 = F128(rom0 & (2 ** 64 - 1), rom0 >> 64)
    w, n = C.c_uint32(), C.c_uint32()
    args = (C.cast(arr, C.c_void_p), len(ops), program_id, commit, C.cast(sec, C.c_void_p), len(secret_args),
            C.cast(ma, C.c_void_p), len(main_args), C.byref(r0))
    rc = lib.zkl_build_trace(*args, None, None, C.byref(w), C.byref(n))
    if rc != 0:
        raise ZklError(rc, "build_trace: invalid program")
    trace = (F128 * (w.value * n.value))()
    pi = AirPublicInputs()
    rc = lib.zkl_build_trace(*args, C.cast(trace, C.c_void_p), C.byref(pi), C.byref(w), C.byref(n))
    if rc != 0:
        raise ZklError(rc, "build_trace: invalid program")
    return trace, pi, w.value, n.value


def rom_acc_from_program(ops, program_id: bytes):
    """romacc::rom_acc_from_program (romacc.rs:22-80) through zkl_rom_acc_from_program: 3 ints."""
    lib = load_library()
    arr = (ZklOp * len(ops))(*ops)
    out = (F128 * 3)()
    rc = lib.zkl_rom_acc_from_program(C.cast(arr, C.c_void_p), len(ops), _id32("program_id", program_id), out)
    if rc != 0:
        raise ZklError(rc, "rom_acc_from_program: invalid program")
    return [e.lo | (e.hi << 64) for e in out]


def plan_segments(n_ops: int, max_rows: int = 1 << 12):
    """WinterfellSegmentPlanner::plan_segments (segment_planner.rs:93-276): [(r_start, r_end)]."""
    lib = load_library()
    k = C.c_uint32()
    if lib.zkl_plan_segments(n_ops, max_rows, None, None, 0, C.byref(k)):
        raise ZklError(-1, "plan_segments: invalid arguments")
    a, b = (C.c_uint32 * k.value)(), (C.c_uint32 * k.value)()
    if lib.zkl_plan_segments(n_ops, max_rows, a, b, k.value, C.byref(k)):
        raise ZklError(-1, "plan_segments: invalid arguments")
    return list(zip(a, b))


def slice_segment(full, width: int, n_rows: int, ops, pi: AirPublicInputs, r_start: int, r_end: int):
    """prove_segment's trace + AirPublicInputs for rows [r_start, r_end) of a build_trace trace
    (zkl_slice_segment): (trace, pi, width, state_in_hash, state_out_hash)."""
    lib = load_library()
    arr = (ZklOp * len(ops))(*ops)
    w = C.c_uint32()
    args = (C.cast(full, C.c_void_p), width, n_rows, C.cast(arr, C.c_void_p), len(ops), C.byref(pi), r_start, r_end)
    rc = lib.zkl_slice_segment(*args, None, None, C.byref(w), None, None)
    if rc:
        raise ZklError(rc, "slice_segment: invalid segment")
    m = r_end - r_start
    t = (F128 * (w.value * m))()
    spi = AirPublicInputs()
    sin, sout = (C.c_uint8 * 32)(), (C.c_uint8 * 32)()
    rc = lib.zkl_slice_segment(*args, C.cast(t, C.c_void_p), C.byref(spi), C.byref(w), sin, sout)
    if rc:
        raise ZklError(rc, "slice_segment: invalid segment")
    return t, spi, w.value, bytes(sin), bytes(sout)


class Program:
    """A program executed once for per-segment trace building (zkl_program_new): what
    prove_segment's input side gives (prove.rs:1057-1134 over build_full_trace + slice,
    vm/trace/mod.rs:316-524) segment by segment, without the full trace in memory.
    `segment(r_start, r_end)` -> (trace, pi, width, state_in_hash, state_out_hash), bit for bit
    slice_segment(build_trace(..)); `width` / `n_rows` are the full trace's shape."""

    def __init__(self, ops, program_id: bytes, program_commitment: bytes | None = None, secret_args=(),
                 main_args=(), rom0: int = 0):
        self.lib = load_library()
        program_id = _id32("program_id", program_id)
        commit = _id32("program_commitment", program_commitment if program_commitment is not None else program_id)
        arr = (ZklOp * len(ops))(*ops)
        sec = (C.c_uint64 * max(1, len(secret_args)))(*secret_args)
        ma = _vm_args(list(main_args))
        r0 = F128(rom0 & (2 ** 64 - 1), rom0 >> 64)
        w, n = C.c_uint32(), C.c_uint32()
        self.ptr = C.c_void_p()
        rc = self.lib.zkl_program_new(C.cast(arr, C.c_void_p), len(ops), program_id, commit,
                                      C.cast(sec, C.c_void_p), len(secret_args), C.cast(ma, C.c_void_p),
                                      len(main_args), C.byref(r0), C.byref(self.ptr), C.byref(w), C.byref(n))
        if rc != 0:
            raise ZklError(rc, "Program: invalid program")
        self.width, self.n_rows, self.n_ops = w.value, n.value, len(ops)

    def segment_width(self, r_start: int, r_end: int) -> int:
        w = C.c_uint32()
        rc = self.lib.zkl_build_segment_trace(self.ptr, r_start, r_end, None, None, C.byref(w), None, None)
        if rc:
            raise ZklError(rc, "build_segment_trace: invalid segment")
        return w.value

    def segment_into(self, r_start: int, r_end: int, out_ptr: int):
        """Writes the segment trace to out_ptr (host memory of width x rows f128):
        (pi, width, state_in_hash, state_out_hash)."""
        w = C.c_uint32()
        spi = AirPublicInputs()
        sin, sout = (C.c_uint8 * 32)(), (C.c_uint8 * 32)()
        rc = self.lib.zkl_build_segment_trace(self.ptr, r_start, r_end, C.c_void_p(out_ptr), C.byref(spi),
                                              C.byref(w), sin, sout)
        if rc:
            raise ZklError(rc, "build_segment_trace: invalid segment")
        return spi, w.value, bytes(sin), bytes(sout)

    def segment(self, r_start: int, r_end: int):
        w = self.segment_width(r_start, r_end)
        t = (F128 * (w * (r_end - r_start)))()
        spi, w, sin, sout = self.segment_into(r_start, r_end, C.addressof(t))
        return t, spi, w, sin, sout

    def close(self):
        if self.ptr:
            self.lib.zkl_program_free(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
