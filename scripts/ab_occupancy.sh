#!/bin/bash
# Trace-builder GPU tests, then hashing throughput of the default build vs occupancy variants
# (tools/build_variant.sh w12 "-DPM_WAVES_CFG=12", w12wide "... -DPM_WIDE_CFG=1")
set -u
out=gpurun_out/ab_occ
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_trace_builder.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/tb.log 2>&1 || { echo "trace builder gpu tests failed"; tail -30 $out/tb.log; exit 1; }
tail -3 $out/tb.log
for v in w12 w12wide; do
  ZKL_HIP_LIB=zk-lisp_amd/build/var/libzkl_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "matrix_core or permute" > $out/par_$v.log 2>&1 || { echo "variant $v parity failed"; tail -20 $out/par_$v.log; exit 1; }
  tail -1 $out/par_$v.log
done
for i in 1 2; do
  echo "default: $(timeout -k 10 120 python3 tools/hashbench.py --reps 3 --only rows,comp,tree)" || exit 1
  for v in w12 w12wide; do
    echo "$v: $(ZKL_HIP_LIB=zk-lisp_amd/build/var/libzkl_hip_$v.so timeout -k 10 120 python3 tools/hashbench.py --reps 3 --only rows,comp,tree)" || exit 1
  done
done
