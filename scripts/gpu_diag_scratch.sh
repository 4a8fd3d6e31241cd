#!/bin/bash
# scratch-memory hypothesis for the stalled steps: the stalling build (ab_mixA) under ROCr scratch
# settings, and this tree's scratch-free coset inversion
set -u
root=$(pwd)
out=$root/gpurun_out/${1:-scr}
mkdir -p $out
run() { local dir=$1 name=$2; shift 2
  (cd $dir && env "$@" timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 > $out/$name.json 2> $out/$name.err) || { echo "$name rc=$?"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['ms_per_step'], d['call_ms_each_step'])"; }
for i in 1 2; do
  run ab_mixA old_default_$i A=1
  run ab_mixA old_noreclaim_$i HSA_NO_SCRATCH_RECLAIM=1
  run ab_mixA old_single4g_$i HSA_SCRATCH_SINGLE_LIMIT=4294967296
  run . new_$i A=1
done
