#!/bin/bash
# matrix-core permutation: parity tests, then stage throughput of both permutation forms
set -u
out=gpurun_out/pm
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "permute or matrix_core" > $out/tests.log 2>&1
rc=$?
tail -25 $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc, stopping"; exit $rc; fi
timeout -k 10 300 python -u tools/hashbench.py --log-rows 20 --reps 3 > $out/hashbench.json 2> $out/hashbench.err
rc2=$?
cat $out/hashbench.json; tail -5 $out/hashbench.err
exit $(( rc != 0 ? rc : rc2 ))
