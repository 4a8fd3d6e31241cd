#!/bin/bash
# GPU-box check without profiling: full gpu test suite + one bench line
set -u
out=gpurun_out/${1:-quick}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
