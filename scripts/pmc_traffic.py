#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch for bench.py's `roofline.traffic`: from a pmc_summary.json
of scripts/pmc_summary.py (keys "<kernel> grid=<g> #<k>"), the second dispatch of each kernel
(steady state; the first if there is one only), FETCH_SIZE x2 (gfx950) + WRITE_SIZE.
  python3 scripts/pmc_traffic.py gpurun_out/<tag>/pmc_summary.json "note" > profiles/rNN/pmc_traffic.json"""
import json
import re
import sys


def main():
    d = json.load(open(sys.argv[1]))
    best = {}
    for k, v in d.items():
        m = re.match(r"^(.*) grid=\d+ #(\d+)$", k)
        if not m or v.get("hbm_bytes") is None:
            continue
        name = m.group(1).replace("zkl::", "")
        rank = int(m.group(2))
        cur = best.get(name)
        # prefer dispatch #2, else the lowest index seen
        if cur is None or (rank == 2) or (cur[0] != 2 and rank < cur[0]):
            best[name] = (rank, int(v["hbm_bytes"]))
    out = {"_note": sys.argv[2] if len(sys.argv) > 2 else "", "per_kernel": {k: v[1] for k, v in sorted(best.items())}}
    row = out["per_kernel"].get("hash_rows_pm_kernel<0, false>")
    if row is not None:
        out["hash_rows_pm_kernel<0>"] = row
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
