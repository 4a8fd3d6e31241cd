"""Host-side check of the device Montgomery helpers (kernels.hip: redc, mac5, mont_mul,
mont_cube) against u128 reference arithmetic: tools/mont_check.hip is compiled for the
host and run (no GPU needed).  Covers lazily-reduced limbs < 2^27 and the 12-term MDS
accumulation at maximal limb values."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_montgomery_helpers(tmp_path):
    build = os.path.join(ROOT, "zk-lisp_amd", "build")
    objs = [os.path.join(build, f) for f in ("host_hash.o", "host_poseidon_ifma.o", "air_host.o")]
    if not all(os.path.exists(o) for o in objs):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "zk-lisp_amd")], check=True)
    obj = tmp_path / "mont_check.o"
    exe = tmp_path / "mont_check"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17", "-c",
                    os.path.join(ROOT, "tools", "mont_check.hip"), "-o", str(obj)], check=True)
    subprocess.run([HIPCC, "--offload-arch=gfx950", str(obj), *objs, "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr
