#!/usr/bin/env python3
"""Per-dispatch timeline of one headline proof from a rocprofv3 --kernel-trace CSV: the proof
that contains the next-to-last trace row hash (hash_rows_pm_kernel<0>), from the first kernel
after the previous proof's query gather to its own gather.  Prints every dispatch (start, duration,
idle gap before it), then per-kernel totals, busy time, idle time and span.
  python3 tools/ktrace_proof.py run_kernel_trace.csv"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"].split("(")[0].replace("zkl::", "").replace("void ", "")
    gathers = [i for i, r in enumerate(rows) if name(r).startswith("gather_kernel")]
    if len(gathers) < 2:
        raise SystemExit("need two proofs in the trace")
    a, b = gathers[-3] + 1 if len(gathers) >= 3 else gathers[-2] + 1, gathers[-2]
    seg = rows[a:b + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    prev = int(rows[a - 1]["End_Timestamp"])
    lead_gap = (t0 - prev) / 1e3
    gaps = busy = 0
    per = collections.defaultdict(lambda: [0, 0.0])
    print(f"idle before the proof's first kernel (previous gather end -> first kernel): {lead_gap:.1f} us")
    prev = t0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = max(s - prev, 0)
        gaps += gap
        busy += e - s
        prev = max(prev, e)
        per[name(r)][0] += 1
        per[name(r)][1] += (e - s) / 1e3
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap {gap / 1e3:6.1f}  {name(r)[:70]}")
    print("---- per kernel (us)")
    for k, (n, us) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{us:10.1f} us {n:4d}x  {k}")
    print(f"busy {busy / 1e6:.3f} ms  gaps {gaps / 1e6:.3f} ms + lead {lead_gap / 1e3:.3f} ms  span {(prev - t0) / 1e6:.3f} ms  launches {len(seg)}")


if __name__ == "__main__":
    main()
