#!/bin/bash
# Round-2 GPU check: GPU test suite, default bench line, 2-rank launcher rehearsal on one GPU.
# Usage (repo root on the box): bash scripts/gpu_r02.sh [tag]
set -u
out=gpurun_out/${1:-r02}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
ZKL_BENCH_DEVICE=0 timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 > $out/bench_2rank_1gpu.json 2> $out/bench2.err || { echo "2-rank bench failed rc=$?"; tail -20 $out/bench2.err; exit 1; }
cat $out/bench_2rank_1gpu.json
