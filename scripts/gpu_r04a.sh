#!/bin/bash
# Round-4 first GPU pass: the real-program tests (rollup-bench / fib-2pow16-log-n, both plans,
# both aggregation modes), the 64-segment chain test with the proof dump for the 64-child
# reference-mode golden, and a short bench with the real-program line.
# Usage (repo root on the box): bash scripts/gpu_r04a.sh [tag]
set -u
root=$(pwd)
out=$root/gpurun_out/${1:-r04a}
mkdir -p $out
export ZKL_DUMP_CHAIN=$out/chain
timeout -k 10 900 python -u -m pytest tests/test_programs.py "tests/test_gpu_parity.py::test_chain_64_segments_and_aggregation_match_goldens" \
  -m gpu -x -v --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -60 $out/pytest_gpu.log; exit 1; }
tail -8 $out/pytest_gpu.log
unset ZKL_DUMP_CHAIN
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --c3-segments 0 --host-steps 0 --c5-log-n 0 \
  > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -20 $out/bench.err; cat $out/bench.json; exit 1; }
python -c "import json,sys; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['parity']['status']); print(json.dumps(d.get('real_program')))"
