#!/usr/bin/env python3
"""Timeline of the last proof in a rocprofv3 --kernel-trace CSV (scripts/ktrace.sh):
per-dispatch start/duration/gap, then totals per kernel name.
  python tools/ktrace_view.py gpurun_out/ktrace/kt/run_kernel_trace.csv [--list]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "scale_bitrev" in r["Kernel_Name"]]
    seg = rows[idx[-1] - 3:]
    t0 = int(seg[0]["Start_Timestamp"])
    prev = t0
    gaps = busy = 0
    per = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("zkl::", "").replace("void ", "")
        gap = s - prev
        gaps += max(gap, 0)
        busy += e - s
        prev = max(prev, e)
        per[name][0] += 1
        per[name][1] += (e - s) / 1e3
        if "--list" in sys.argv:
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap {gap / 1e3:6.1f}  {name[:60]}")
    for k, (n, us) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{us / 1e3:8.3f} ms  {n:4d}x  {k}")
    print(f"busy {busy / 1e6:.3f} ms  gaps {gaps / 1e6:.3f} ms  span {(prev - t0) / 1e6:.3f} ms  launches {len(seg)}")


if __name__ == "__main__":
    main()
