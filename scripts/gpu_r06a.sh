#!/bin/bash
# round 6: GPU parity suite on the pruned permutations, then A/B against the round-5 library
set -u
out=gpurun_out/r06a
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu rc=$?"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
bash scripts/ab_r06.sh r06a/ab abvar/base.so abvar/p3.so abvar/p1.so
