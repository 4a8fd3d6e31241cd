#!/bin/bash
# Poseidon-block evaluator occupancy A/B on the real-program line (rollup-bench, 212 columns)
set -u
out=$(pwd)/gpurun_out/${1:-cepose}
mkdir -p $out
run() { local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 8 > $out/$name.json 2> $out/$name.err || { echo "$name rc=$?"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); rp=d['real_program']; print('$name', rp['ms_per_proof'], rp['parity'], rp['kernel_ms_per_family_untimed_step']['constraint_eval'])"; }
for i in 1 2; do
  run base_$i A=1
  run w3_$i ZKL_HIP_LIB=$(pwd)/var_libs/libzkl_hip_cepose3.so
  run w4_$i ZKL_HIP_LIB=$(pwd)/var_libs/libzkl_hip_cepose4.so
done
