#!/bin/bash
# A/B: HSA_ENABLE_SDMA=0 (every copy as a blit kernel) against the stalled steps, after a warm-up
set -u
out=$(pwd)/gpurun_out/${1:-sdma}
mkdir -p $out
timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/w.json 2> $out/w.err || exit 1
for i in 1 2 3; do
  for sd in 0 1; do
    HSA_ENABLE_SDMA=$sd timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/b${sd}_$i.json 2> $out/b${sd}_$i.err || { echo "rc=$?"; tail -5 $out/b${sd}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/b${sd}_$i.json')); print('sdma=$sd run $i', d['ms_per_step'], d['call_ms_each_step'])"
  done
done
