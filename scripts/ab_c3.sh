#!/bin/bash
# A/B of the configs[2] in-GPU pipeline (8 segments, 1/2/4 contexts in flight): default vs
# variant libraries (*.so) and environment settings (NAME=VALUE), one bench run each.
#   bash scripts/ab_c3.sh tag [var.so | NAME=VALUE | "NAME=VALUE var.so"] ...
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --c5-log-n 0 --c3-inflight 1,2,4,6"
run() {  # name, then env assignments / library
  local n=$1; shift
  ( for a in "$@"; do case $a in *.so) export ZKL_HIP_LIB=$a ;; *) export "$a" ;; esac; done
    timeout -k 10 300 python3 $B > $out/$n.json 2> $out/$n.err ) || { echo "$n rc=$?"; tail -5 $out/$n.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['c3_in_gpu_pipeline']['segment_proofs_per_s_by_inflight'])" $out/$n.json $n
}
run default
i=0
for v in "$@"; do i=$((i+1)); run v$i $v; echo "  v$i = $v"; done
