#!/usr/bin/env python3
"""Per-kernel scratch / VGPR / spill report of a HIP translation unit (hipcc
-Rpass-analysis=kernel-resource-usage).  Product kernels need no scratch (a kernel with a private
segment makes the runtime allocate the queue's scratch memory on dispatch) except the
constraint evaluators listed in tests/test_abi.py (SCRATCH_ALLOWED), which checks the shipped
library with tools/kernel_resources.py.

    python tools/scratch_check.py zk-lisp_amd/csrc/kernels.hip [extra hipcc flags]
"""
import re
import subprocess
import sys


def report(src, flags=()):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-function",
           "-Rpass-analysis=kernel-resource-usage", *flags, "-c", src, "-o", "/dev/null"]
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    out, cur = {}, None
    for line in err.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur:
            out[cur][m.group(1).split(" [")[0]] = int(m.group(2))
    return out


if __name__ == "__main__":
    r = report(sys.argv[1], sys.argv[2:])
    bad = 0
    for k, v in r.items():
        if v.get("ScratchSize", 0) or v.get("VGPRs Spill", 0) or len(sys.argv) > 1 and "-v" in sys.argv:
            print(f"{k[:90]:90s} {v}")
        bad += v.get("ScratchSize", 0) > 0
    print(f"{len(r)} kernels, {bad} with scratch")
