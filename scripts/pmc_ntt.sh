#!/bin/bash
# SQ counters of the DIT NTT passes (hashbench --only ntt: 204 x 2^20, all 20 stages), both forms
set -u
out=$PWD/gpurun_out/${1:-pmc_ntt}
mkdir -p $out
export TMPDIR=/tmp
root=$PWD
cd /tmp
for mode in lazy classic; do
  if [ $mode = classic ]; then export ZKL_NTT=classic; else unset ZKL_NTT; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU -d $out/${mode}_p1 -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 --only ntt > $out/${mode}_hb1.json 2> $out/${mode}_p1.err || { echo "p1 rc=$?"; tail -5 $out/${mode}_p1.err; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $out/${mode}_p2 -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 --only ntt > $out/${mode}_hb2.json 2> $out/${mode}_p2.err || { echo "p2 rc=$?"; tail -5 $out/${mode}_p2.err; exit 1; }
done
unset ZKL_NTT
timeout -k 10 60 python3 $root/tools/hashbench.py --reps 3 --only ntt > $out/lazy_time.json
ZKL_NTT=classic timeout -k 10 60 python3 $root/tools/hashbench.py --reps 3 --only ntt > $out/classic_time.json
cat $out/lazy_time.json $out/classic_time.json
python3 - <<'PY' "$out"
import csv, glob, sys, collections
out = sys.argv[1]
for mode in ("lazy", "classic"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{out}/{mode}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        if "ntt" in k:
            print(mode, k[:50], {c: f"{x:.4e}" for c, x in sorted(v.items())})
PY
