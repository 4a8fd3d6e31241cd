#!/usr/bin/env python3
"""Summarise the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of scripts/pmc.sh: per kernel
name, the mean counter value per dispatch, converted to bytes with the gfx950 correction
of MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of wide streaming reads, so it
is doubled; WRITE_SIZE is taken as is).  Counter unit: KiB (rocprofv3 FETCH_SIZE /
WRITE_SIZE are kilobytes)."""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(list)
    rows = []
    for f in files:
        rows += [r for r in csv.DictReader(open(f)) if r.get("Counter_Name") == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    seen = collections.Counter()
    for row in rows:  # key: (kernel, grid, k-th dispatch of that kernel+grid within the run)
        name = row["Kernel_Name"].split("(")[0].replace("void ", "")
        g = row.get("Grid_Size", row.get("Grid_Size_X", ""))
        seen[(name, g)] += 1
        acc[(name, g, seen[(name, g)])].append(float(row["Counter_Value"]))
    return acc


def main():
    out = sys.argv[1]
    fetch = per_kernel(os.path.join(out, "pmc_fetch"), "FETCH_SIZE")
    write = per_kernel(os.path.join(out, "pmc_write"), "WRITE_SIZE")
    res = {}
    for key in sorted(set(fetch) | set(write)):
        f = fetch.get(key, [])
        w = write.get(key, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        res[f"{key[0]} grid={key[1]} #{key[2]}"] = {
            "dispatches": max(len(f), len(w)),
            "fetch_kib_raw": fk,
            "write_kib": wk,
            "hbm_bytes": (2 * fk * 1024 if fk is not None else 0) + (wk * 1024 if wk is not None else 0),
        }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
