#!/bin/bash
# trace row hash under scheduling variants of the Poseidon translation unit (tools/hashbench.py)
set -u
out=$(pwd)/gpurun_out/${1:-absched}
mkdir -p $out
run() { local name=$1 lib=$2
  if [ -n "$lib" ]; then export ZKL_HIP_LIB=$(pwd)/var_libs/$lib; else unset ZKL_HIP_LIB; fi
  timeout -k 10 200 python3 tools/hashbench.py --reps 5 --only rows,comp,tree > $out/$name.json 2> $out/$name.err || { echo "$name rc=$?"; tail -5 $out/$name.err; exit 1; }
  echo "$name $(cat $out/$name.json)"; }
for i in 1 2; do
  run base_$i ""
  run noiglp_$i libzkl_hip_noiglp.so
  run trackers_$i libzkl_hip_trackers.so
  run defsched_$i libzkl_hip_defsched.so
done
