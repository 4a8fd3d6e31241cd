#!/usr/bin/env python3
"""Per-kernel resources of a built HIP shared library, read from its device code objects: the
.hip_fatbin section holds one offload bundle per translation unit; each gfx950 code object's
AMDGPU metadata gives .private_segment_fixed_size (scratch bytes per lane), .vgpr_count and
.vgpr_spill_count.  Product kernels must need no scratch: a kernel with a private segment makes the
runtime allocate the queue's scratch memory on dispatch.

    python tools/kernel_resources.py [zk-lisp_amd/zkl_hip/libzkl_hip.so]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernel_resources(lib):
    """{mangled kernel name: {"scratch": int, "vgpr": int, "spill": int}} over every bundle."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fb.bin")
        # an explicit output file: without one objcopy rewrites `lib` in place (which also breaks a
        # process that has it mapped)
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", lib, os.path.join(td, "discard.so")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for k, a in enumerate(starts):
            b = starts[k + 1] if k + 1 < len(starts) else len(data)
            part = os.path.join(td, f"b{k}.bin")
            open(part, "wb").write(data[a:b])
            co = os.path.join(td, f"b{k}.co")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
            cur = None
            for line in notes.splitlines():
                m = re.match(r"\s+\.name:\s+(\S+)", line)
                if m and m.group(1).startswith("_Z"):
                    cur = m.group(1)
                    out[cur] = {}
                    continue
                m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_count|vgpr_spill_count):\s+(\d+)", line)
                if m and cur:
                    key = {"private_segment_fixed_size": "scratch", "vgpr_count": "vgpr",
                           "vgpr_spill_count": "spill"}[m.group(1)]
                    out[cur][key] = int(m.group(2))
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                            "zk-lisp_amd", "zkl_hip", "libzkl_hip.so")
    res = kernel_resources(lib)
    for k, v in sorted(res.items()):
        flag = " <-- scratch" if v.get("scratch") or v.get("spill") else ""
        print(f"{k[:100]:100s} vgpr {v.get('vgpr', '?'):>4} spill {v.get('spill', '?'):>3} scratch {v.get('scratch', '?'):>4}{flag}")
    print(f"{len(res)} kernels, {sum(1 for v in res.values() if v.get('scratch'))} with scratch")
