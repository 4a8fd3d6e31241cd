#!/bin/bash
# round 5: the shader clock while the row hash runs -- GRBM_GUI_ACTIVE per dispatch (summed over
# the 8 XCDs) over the dispatch's duration from the kernel trace of the same pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$PWD/gpurun_out/r05o
mkdir -p $out
export TMPDIR=/tmp
root=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p -o run --output-format csv -- python3 $root/tools/hashbench.py --reps 2 --only rows,comp,tree,ntt > $out/hb.json 2> $out/p.err || { echo "pass rc=$?"; tail -5 $out/p.err; exit 1; }
cd $root
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
cc = {}
for f in glob.glob(out + "/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        cc.setdefault((r["Dispatch_Id"], r["Kernel_Name"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
dur = {}
for f in glob.glob(out + "/p/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = collections.defaultdict(list)
for (d, k), v in cc.items():
    if d in dur and dur[d] > 20e-6:
        agg[k.split("(")[0][:60]].append(v.get("GRBM_GUI_ACTIVE", 0) / 8 / dur[d] / 1e6)
for k, v in sorted(agg.items()):
    print(f"{k:60s} n {len(v):3d} MHz (GRBM_GUI_ACTIVE/8/duration) median {sorted(v)[len(v)//2]:7.0f}")
PY
