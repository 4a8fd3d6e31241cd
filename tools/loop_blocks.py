#!/usr/bin/env python3
"""Instruction counts of every block of one loop (LLVM's "Loop: Header=" block annotations)
in a hipcc -save-temps .s file: the whole loop body, not only the straight-line range between
a label and its back edge (tools/isa_hist.py), so rotated loops with branches count fully.
  python tools/loop_blocks.py poseidon-hip-amdgcn-amd-amdhsa-gfx950.s merkle_top_kernel [depth]"""
import collections
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    key = sys.argv[2]
    depth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    m = re.search(r"^(_Z\S*" + re.escape(key) + r"\S*):", s, re.M)
    end = s.index(".Lfunc_end", m.start())
    lines = s[m.start():end].split("\n")
    blocks, cur = [], None
    for i, l in enumerate(lines):
        if re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", l) or re.match(r"^\.LBB\d+_\d+:", l):
            cur = {"label": l.split(":")[0], "ann": "", "ins": collections.Counter()}
            blocks.append(cur)
            continue
        if cur is None:
            continue
        t = l.strip()
        if t.startswith(";"):
            cur["ann"] += t
            continue
        if not t or t.startswith("."):
            continue
        cur["ins"][t.split()[0]] += 1
    headers = collections.defaultdict(list)
    for b in blocks:
        mm = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", b["ann"])
        if mm and int(mm.group(2)) == depth:
            headers[mm.group(1)].append(b)
        elif b["label"].startswith(".L") and f"Depth={depth}" in b["ann"] and "Loop Header" in b["ann"]:
            headers[b["label"][2:]].append(b)
    for h, bl in headers.items():
        c = collections.Counter()
        for b in bl:
            c.update(b["ins"])
        valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
        print(f"loop {h}: {len(bl)} blocks, total {sum(c.values())}, valu {valu}, "
              f"mad {c['v_mad_u64_u32'] + c['v_mad_i64_i32']}, ds {sum(v for k, v in c.items() if k.startswith('ds_'))}")


if __name__ == "__main__":
    main()
