"""C-ABI library checks that need no GPU: libzkl_hip.so loads, exports every function
declared in include/zkl_hip.h, and its host-side helpers agree with the oracle."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zkl_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zkl_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_all_symbols():
    import zkl_hip
    lib = zkl_hip.load_library()
    names = declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), f"missing export {n}"


def test_abi_version():
    import zkl_hip
    assert zkl_hip.load_library().zkl_hip_abi_version() == 1


def test_pinned_bytes_query_needs_no_device():
    import zkl_hip
    cur, peak = zkl_hip.pinned_bytes()
    assert 0 <= cur <= peak


def test_build_carries_only_default_tuning_values():
    """no timing probe or losing variant is compiled into the shipped library;
    the Poseidon translation unit is built with the default scheduler."""
    import zkl_hip
    lib = zkl_hip.load_library()
    lib.zkl_hip_build_config.restype = C.c_char_p
    cfg = dict(kv.split("=") for kv in lib.zkl_hip_build_config().decode().split(";"))
    assert cfg == {"PM_WAVES": "8", "PM_WIDE": "0", "PM_ROW_WAVES": "8", "PM_IGLP": "0", "TAIL_PRIO": "0",
                   "PW_MAX_ITEMS": "2048", "PM_ROW_BIG": "0", "POSEIDON_SCHED": "default", "NTT_ELEMS": "1024",
                   "NTT_THREADS": "256", "CE_WAVES": "3", "CE_POSE_WAVES": "3", "DEEP_PTS": "2",
                   "DEEP_COLS": "4", "PM_PRUNE": "3", "TOP_LDS": "1", "TOP_WAVES": "4", "CE_GROUPS": "31",
                   "CE_DOT": "0", "CE_BRANCHFREE": "0"}


def test_select_partitions():
    import zkl_hip
    for w, n, exp in [(204, 1 << 12, (1, 16)), (204, 1 << 14, (2, 16)), (204, 1 << 16, (4, 16)),
                      (204, 1 << 18, (8, 16)), (204, 1 << 20, (16, 16)), (31, 16, (1, 8))]:
        assert zkl_hip.select_partitions_for_trace(w, n) == exp


WIDTHS = {0: 204, 1: 204, 2: 212, 3: 212, 4: 211, 5: 211, 6: 219, 7: 219}


@pytest.mark.parametrize("flags", range(8))
@pytest.mark.parametrize("log_n", [5, 6, 8, 10, 12])
def test_product_tracegen_matches_oracle(oracle, log_n, flags):
    """Generator flags: 1 sponge, 2 RAM, 4 Merkle (needs log_n >= 8)."""
    import zkl_hip
    if flags & 4 and log_n < 8:
        with pytest.raises(zkl_hip.ZklError):
            zkl_hip.synth_vm_segment(0x5EED0001 + log_n, log_n, flags)
        return
    t1, pi1, w1 = zkl_hip.synth_vm_segment(0x5EED0001 + log_n, log_n, flags)
    t2, pi2, w2 = oracle.synth_segment(0x5EED0001 + log_n, log_n, flags)
    assert w1 == w2 == WIDTHS[flags]
    assert bytes(t1) == bytes(t2)
    assert bytes(pi1) == bytes(pi2)


def test_init_without_gpu_fails_cleanly():
    import zkl_hip
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(zkl_hip.ZklError):
        zkl_hip.Context(0)


def _req(log_n=6, **kw):
    import zkl_hip
    t, pi, w = zkl_hip.synth_vm_segment(0x5EED0300, max(log_n, 5))
    opts = zkl_hip.proof_options(w, 1 << max(log_n, 5), queries=8, grind=0)
    for k, v in kw.items():
        if hasattr(opts, k):
            setattr(opts, k, v)
    if "n_main_slots" in kw:
        pi.n_main_slots = kw["n_main_slots"]
    return w - kw.get("width_delta", 0), 1 << log_n, pi, opts


def test_check_request_accepts_valid():
    import zkl_hip
    for log_n in (5, 8, 14, 16):
        w, n, pi, opts = _req(log_n)
        zkl_hip.check_request(w, n, pi, opts)


@pytest.mark.parametrize("change,msg", [
    (dict(log_n=4), "power of two >= 32"),
    (dict(blowup_factor=4), "blowup factor below"),
    (dict(blowup_factor=12), "power of two"),
    (dict(blowup_factor=1), "power of two"),
    (dict(num_queries=0), "num_queries"),
    (dict(num_queries=256), "num_queries"),
    (dict(field_extension=2), "FieldExtension::None"),
    (dict(fri_folding_factor=4), "folding factor"),
    (dict(fri_remainder_max_degree=2), "fri_remainder_max_degree"),
    # the verifier's bound (remainder degree below the blowup) holds in the prover too
    (dict(blowup_factor=8, fri_remainder_max_degree=15), "below the blowup factor"),
    (dict(batching_constraints=1), "Linear"),
    (dict(batching_deep=1), "Linear"),
    (dict(num_partitions=0), "num_partitions"),
    (dict(num_partitions=17), "num_partitions"),
    (dict(num_partitions=64), "num_partitions"),
    (dict(hash_rate=0), "hash_rate"),
    (dict(hash_rate=256), "hash_rate"),
    (dict(hash_rate=257), "hash_rate"),
    (dict(grinding_factor=33), "grinding_factor"),
    (dict(grinding_factor=65), "grinding_factor"),
    (dict(blowup_factor=256), "at most 128"),
    (dict(n_main_slots=9), "ZKL_MAX_MAIN_SLOTS"),
    (dict(n_main_slots=1000), "ZKL_MAX_MAIN_SLOTS"),
    (dict(width_delta=1), "width"),
])
def test_check_request_rejections(change, msg):
    """Each request the prover refuses is refused on the host, before any device work, with
    ZKL_E_INVALID and a message (n_main_slots read past main_slots, unchecked
    num_partitions / hash_rate)."""
    import zkl_hip
    w, n, pi, opts = _req(**change)
    with pytest.raises(zkl_hip.ZklError, match=msg) as ei:
        zkl_hip.check_request(w, n, pi, opts)
    assert ei.value.code == -1


def test_row_digest_rule_switch():
    import zkl_hip
    lib = zkl_hip.load_library()
    assert lib.zkl_hip_row_digest_rule() == 0
    with zkl_hip.row_digest_rule(1):
        assert lib.zkl_hip_row_digest_rule() == 1
    assert lib.zkl_hip_row_digest_rule() == 0
    assert lib.zkl_hip_set_row_digest_rule(2) == -1


def test_ntt_mode_switch_bounds():
    """zkl_hip_set_ntt_mode: 0 canonical, 1 lazy (default); the matrix-core NTT (mode 2, measured
    slower in round 3) is no longer built."""
    import zkl_hip
    lib = zkl_hip.load_library()
    try:
        for mode in (0, 1):
            assert lib.zkl_hip_set_ntt_mode(mode) == 0
        assert lib.zkl_hip_set_ntt_mode(2) == -1
        assert lib.zkl_hip_set_ntt_mode(3) == -1
        assert lib.zkl_hip_set_ntt_mode(-1) == -1
    finally:
        lib.zkl_hip_set_ntt_mode(1)


# Kernels allowed a private segment (scratch), each measured faster than its scratch-free form:
# the constraint evaluators at 3 waves per SIMD spill (1.57 -> 1.40 ms per headline proof,
# DESIGN.md §5; 3.42 -> 3.33 ms of Poseidon-block evaluation per rollup-bench proof,
# profiles/r04/ab_cepose.json), and the Poseidon-block part keeps a stack object at any occupancy.
# The runtime allocates a queue's scratch at the first dispatch that needs it and keeps it; the
# round-4 stall study found scratch settings irrelevant (profiles/r04/stalls.md, "scr1").
SCRATCH_ALLOWED = ("constraint_eval_kernel", "constraint_eval_pose_kernel", "constraint_eval_pose_part_kernel")


def test_only_listed_kernels_need_scratch():
    """every kernel of the shipped library is scratch-free except the listed
    evaluator kernels (read from the device code objects' metadata, tools/kernel_resources.py)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_resources import kernel_resources
    import zkl_hip
    res = kernel_resources(zkl_hip.LIB_PATH)
    assert len(res) > 40, "device code objects not found"
    bad = [k for k, v in res.items() if (v.get("scratch") or v.get("spill")) and
           not any(a in k for a in SCRATCH_ALLOWED)]
    assert not bad, bad
    assert all(v.get("scratch", 0) == 0 for k, v in res.items() if "pm_kernel" in k or "ntt" in k or "deep" in k)
