#!/bin/bash
# A/B: the round-3 build (ab_r03tree) against this one, interleaved, after a warm-up
set -u
root=$(pwd)
out=$root/gpurun_out/${1:-r03ab}
mkdir -p $out
timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/w.json 2> $out/w.err || exit 1
for i in 1 2 3; do
  (cd ab_r03tree && timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 > $out/r03_$i.json 2> $out/r03_$i.err) || { echo "r03 rc=$?"; tail -5 $out/r03_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/r03_$i.json')); print('r03 run $i', d['ms_per_step'], d['call_ms_each_step'])"
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/r04_$i.json 2> $out/r04_$i.err || exit 1
  python3 -c "import json; d=json.load(open('$out/r04_$i.json')); print('r04 run $i', d['ms_per_step'], d['call_ms_each_step'])"
done
