#!/bin/bash
# GPU-box check: parity tests, a short bench line, a rocprofv3 kernel-trace summary.
# Usage (from the repo root on the box): bash scripts/gpu_check.sh [tag]
set -u
tag=${1:-r01}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
export TMPDIR=/tmp
root=$PWD
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $root/$out/prof -o run --output-format csv -- python3 $root/bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-inflight 1 > $root/$out/prof_bench.json 2> $root/$out/prof.err || { echo "rocprof failed rc=$?"; tail -20 $root/$out/prof.err; exit 1; }
echo done
