#!/bin/bash
# SQ counters per kernel over one headline proof (bench.py --steps 1): one 8-counter pass
#   bash scripts/pmc_sq_proof.sh tag -> gpurun_out/<tag>/{sq/,sq_per_kernel.json}
set -u
root=$PWD
out=$root/gpurun_out/${1:-sqproof}
mkdir -p $out
export TMPDIR=/tmp
B="$root/bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 --programs none"
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $out/sq -o run --output-format csv -- python3 $B > $out/sq.json 2> $out/sq.err || { echo "sq pass rc=$?"; tail -5 $out/sq.err; exit 1; }
cd $root
python3 - <<'PY' "$out"
import csv, glob, sys, collections, json
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in glob.glob(out + "/sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
res = {k: dict(v) for k, v in acc.items()}
json.dump(res, open(out + "/sq_per_kernel.json", "w"), indent=1)
for k, v in sorted(res.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:12]:
    wc = v.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{k[:60]:60s} VALU {v.get('SQ_INSTS_VALU',0):.3e} waves {v.get('SQ_WAVES',0):.0f} wait_inst {v.get('SQ_WAIT_INST_ANY',0)/wc:.3f} wait_any {v.get('SQ_WAIT_ANY',0)/wc:.3f}")
PY
