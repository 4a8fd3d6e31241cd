#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 --kernel-trace rocpd database (rocprofv3's default
output format on this image), in the column layout of its --stats kernel_stats.csv:
Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, plus VGPRs / LDS bytes.

    python tools/rocpd_stats.py gpurun_out/r03a/prof/run_results.db > profiles/r03/kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select s.display_name, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.end - d.start), "
        "max(s.arch_vgpr_count), max(s.accum_vgpr_count), max(d.group_segment_size) "
        "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
        "group by s.display_name order by sum(d.end - d.start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "ArchVGPR",
                "AccumVGPR", "LDSBytes"])
    for name, n, t, mn, mx, vg, ag, lds in rows:
        w.writerow([name, n, t, round(t / n, 1), round(100.0 * t / tot, 3), mn, mx, vg, ag, lds])


if __name__ == "__main__":
    main(sys.argv[1])
