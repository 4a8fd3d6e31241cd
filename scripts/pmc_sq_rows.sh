#!/bin/bash
# SQ counters of the trace row hash (hashbench rows only), two passes (8 SQ counters each):
#   bash scripts/pmc_sq_rows.sh tag -> gpurun_out/<tag>/
set -u
out=$PWD/gpurun_out/${1:-sqrows}
mkdir -p $out
export TMPDIR=/tmp
root=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU -d $out/p1 -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 --only rows > $out/hb1.json 2> $out/p1.err || { echo "pass 1 rc=$?"; tail -5 $out/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p2 -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 --only rows > $out/hb2.json 2> $out/p2.err || { echo "pass 2 rc=$?"; tail -5 $out/p2.err; exit 1; }
python3 - <<'PY' "$out"
import csv, glob, sys, collections, json
out = sys.argv[1]
acc = collections.defaultdict(float)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "hash_rows_pm_kernel<0" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
json.dump(acc, open(out + "/sq_rows.json", "w"), indent=1)
print(json.dumps(acc))
PY
