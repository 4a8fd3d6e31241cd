#!/usr/bin/env python3
"""Per-kernel average duration (us) side by side from rocprofv3 --stats directories."""
import csv
import glob
import sys

cols = []
for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
    rows = {r["Name"].split("(")[0].replace("void ", "").replace("zkl::", ""): r for r in csv.DictReader(open(f[0]))}
    cols.append((d.rstrip("/").split("/")[-1], rows))
names = sorted(set().union(*[set(r) for _, r in cols]), key=lambda n: -float(cols[0][1].get(n, {}).get("TotalDurationNs", 0)))
print(f"{'kernel':44s}" + "".join(f"{c[0]:>14s}" for c in cols))
for n in names[:40]:
    print(f"{n[:44]:44s}" + "".join(f"{float(r[n]['AverageNs']) / 1e3 if n in r else float('nan'):14.1f}" for _, r in cols))
print(f"{'TOTAL ms':44s}" + "".join(f"{sum(float(x['TotalDurationNs']) for x in r.values()) / 1e6:14.2f}" for _, r in cols))
