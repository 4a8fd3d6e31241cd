#!/bin/bash
# SQ (wave scheduler) counters for the stage kernels: issue vs wait breakdown.
set -u
out=$PWD/gpurun_out/${1:-sq}
mkdir -p $out
export TMPDIR=/tmp
root=$PWD
cd /tmp
timeout -k 10 120 rocprofv3 -L > $out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU -d $out/pmc_sq -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 > $out/hb.json 2> $out/pmc_sq.err || { echo "pmc failed rc=$?"; tail -20 $out/pmc_sq.err; grep -i "sq_" $out/counters.txt | head -80; exit 1; }
python3 - <<'PY' "$out"
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/pmc_sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print(k[:60], {c: f"{x:.3e}" for c, x in sorted(v.items())})
PY
