#!/bin/bash
# A/B of the matrix-core hashing kernels: default build vs a variant library
#   bash scripts/ab_pm.sh <variant .so> [tag]
set -u
var=$1
out=gpurun_out/${2:-ab_pm}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "matrix_core or permute" > $out/tests.log 2>&1
rc=$?
tail -2 $out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 120 python3 tools/hashbench.py --reps 3 --only rows,comp,tree,perm || exit 1
  ZKL_HIP_LIB=$var timeout -k 10 120 python3 tools/hashbench.py --reps 3 --only rows,comp,tree,perm || exit 1
done
