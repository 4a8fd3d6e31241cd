#!/bin/bash
# GPU test suite + smoke on the box: bash scripts/gpu_tests.sh [tag] -> gpurun_out/<tag>/
set -u
out=gpurun_out/${1:-tests}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
cat $out/smoke.log
