#!/bin/bash
# SQ counters of the trace row hash (hashbench rows only) for the shipped library and a variant:
#   bash scripts/pmc_sq_ab.sh tag var_libs/libzkl_hip_X.so -> gpurun_out/<tag>/{base,var}/sq_rows.json
set -u
root=$PWD
tag=${1:-sqab}; var=$root/${2:-var_libs/libzkl_hip_pair.so}
export TMPDIR=/tmp
for which in base var; do
  out=$root/gpurun_out/$tag/$which
  mkdir -p $out
  if [ $which = var ]; then export ZKL_HIP_LIB=$var; else unset ZKL_HIP_LIB; fi
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU -d $out/p1 -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 --only rows > $out/hb1.json 2> $out/p1.err || { echo "$which pass 1 rc=$?"; tail -5 $out/p1.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p2 -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 1 --only rows > $out/hb2.json 2> $out/p2.err || { echo "$which pass 2 rc=$?"; tail -5 $out/p2.err; exit 1; }
  cd $root
  python3 - <<'PY' "$out"
import csv, glob, sys, collections, json
out = sys.argv[1]
acc = collections.defaultdict(float)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "hash_rows_pm_kernel<0" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
json.dump(acc, open(out + "/sq_rows.json", "w"), indent=1)
w = acc.get("SQ_WAVE_CYCLES", 1)
print(out.split("/")[-1], {k: round(v / w, 4) for k, v in acc.items() if k.startswith("SQ_WAIT") or k.startswith("SQ_ACTIVE")},
      "VALU", acc.get("SQ_INSTS_VALU"), "wave_cycles", w)
PY
done
