"""The C++ host mirror of the reference's prover API (include/zkl_hip.hpp: ZkProver, verify_proof,
StepProof, WinterfellBackend, Error) through its test program tests/cpp/host_api_test: request
checks and error mapping without a device, and on the GPU a proof whose bytes equal the CPU
oracle's, verified, wrapped as a zl1 step and aggregated."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "host_api_test")


def _binary():
    if not os.path.exists(BIN):  # host-only g++ build against libzkl_hip.so (zk-lisp_amd/Makefile)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "zk-lisp_amd"), "../tests/cpp/host_api_test"], check=True)
    return BIN


def test_cpp_host_api_cpu():
    r = subprocess.run([_binary(), "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok cpu")


@pytest.mark.gpu
def test_cpp_host_api_gpu_proof_equals_oracle(oracle, tmp_path):
    import zkl_hip
    out = tmp_path / "proof.bin"
    r = subprocess.run([_binary(), "gpu", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = out.read_bytes()
    log_n, n = 8, 1 << 8
    ot, opi, w = oracle.synth_segment(0x5EED0001, log_n)
    opts = zkl_hip.proof_options(w, n, queries=32, grind=8)
    want = oracle.prove(ot, w, n, opi, oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_]))
    assert got == want
