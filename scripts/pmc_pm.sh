#!/bin/bash
# SQ counters of the matrix-core row hash (hashbench --only rows), two passes
set -u
out=$PWD/gpurun_out/${1:-pmc_pm}
mkdir -p $out
export TMPDIR=/tmp
root=$PWD
cd /tmp
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU -d $out/p1 -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 --only rows > $out/hb1.json 2> $out/p1.err || { echo "p1 rc=$?"; tail -5 $out/p1.err; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p2 -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 --only rows > $out/hb2.json 2> $out/p2.err || { echo "p2 rc=$?"; tail -5 $out/p2.err; }
python3 - <<'PY' "$out"
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print(k[:60], {c: f"{x:.4e}" for c, x in sorted(v.items())})
PY
