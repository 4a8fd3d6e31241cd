#!/bin/bash
# A/B of spin-waiting (ZKL_SPIN) against the alternating slow steps, 3 runs each, interleaved
set -u
out=$(pwd)/gpurun_out/${1:-spin}
mkdir -p $out
for i in 1 2 3; do
  for sp in 1 0; do
    ZKL_SPIN=$sp timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/b${sp}_$i.json 2> $out/b${sp}_$i.err || { echo "rc=$?"; tail -5 $out/b${sp}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/b${sp}_$i.json')); print('spin=$sp run $i', d['ms_per_step'], d['call_ms_each_step'])"
  done
done
