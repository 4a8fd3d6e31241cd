#!/bin/bash
# instruction-cache counters of the trace row hash (hashbench rows only), one 8-counter SQ pass:
#   bash scripts/pmc_icache_rows.sh tag -> gpurun_out/<tag>/icache_rows.json
set -u
out=$PWD/gpurun_out/${1:-icache}
mkdir -p $out
export TMPDIR=/tmp
root=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES SQ_INSTS_VALU -d $out/p1 -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 --only rows > $out/hb1.json 2> $out/p1.err || { echo "pass rc=$?"; tail -5 $out/p1.err; exit 1; }
python3 - <<'PY' "$out"
import csv, glob, sys, collections, json
out = sys.argv[1]
acc = collections.defaultdict(float)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "hash_rows_pm_kernel<0" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
json.dump(acc, open(out + "/icache_rows.json", "w"), indent=1)
print(json.dumps(acc))
PY
