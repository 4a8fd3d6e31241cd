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
