#!/bin/bash
# Round-3 GPU check: GPU test suite, default bench line, rocprofv3 kernel stats of a short bench.
# Usage (repo root on the box): bash scripts/gpu_r03.sh [tag] [skip-tests]
set -u
root=$(pwd)
out=$root/gpurun_out/${1:-r03}
mkdir -p $out
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -40 $out/pytest_gpu.log; exit 1; }
  tail -3 $out/pytest_gpu.log
fi
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -20 $out/bench.err; cat $out/bench.json; exit 1; }
cat $out/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $root/bench.py --steps 8 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 > $out/prof_bench.json 2> $out/prof_bench.err || { echo "rocprof failed rc=$?"; tail -20 $out/prof_bench.err; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -3
