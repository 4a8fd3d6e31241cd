#!/usr/bin/env python3
"""Instruction histogram of the innermost loops of one kernel in a hipcc -save-temps .s file.
  python tools/isa_hist.py kernels-hip-amdgcn-amd-amdhsa-gfx950.s <mangled-name-substring>"""
import collections
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    key = sys.argv[2]
    m = re.search(r"^(_Z\S*" + re.escape(key) + r"\S*):", s, re.M)
    start = m.start()
    end = s.index(".Lfunc_end", start)
    lines = s[start:end].split("\n")
    labels = {}
    for i, l in enumerate(lines):
        mm = re.match(r"^(\.LBB\d+_\d+):", l)
        if mm:
            labels[mm.group(1)] = i
    loops = []
    for i, l in enumerate(lines):
        mm = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)", l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
            loops.append((labels[mm.group(1)], i))
    for a, b in loops:
        c = collections.Counter()
        for l in lines[a:b + 1]:
            l = l.strip()
            if not l or l.startswith(";") or l.startswith("."):
                continue
            c[l.split()[0]] += 1
        valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
        mf = sum(v for k, v in c.items() if "mfma" in k)
        print(f"loop lines {a}-{b}: total {sum(c.values())} valu {valu} mfma {mf} ds {sum(v for k, v in c.items() if k.startswith('ds_'))}")
        if len(sys.argv) > 3:
            for k, v in c.most_common(int(sys.argv[3])):
                print("   ", v, k)


if __name__ == "__main__":
    main()
