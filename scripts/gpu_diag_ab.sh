#!/bin/bash
# stalled-step A/B: warm-up, then interleaved runs of the listed trees ("." = this one)
set -u
root=$(pwd)
out=$root/gpurun_out/${1:-ab}; shift
mkdir -p $out
timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/w.json 2> $out/w.err || exit 1
for i in 1 2 3; do
  for t in "$@"; do
    n=$(echo $t | tr -d './'); n=${n:-cur}
    (cd $t && timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 > $out/${n}_$i.json 2> $out/${n}_$i.err) || { echo "$t rc=$?"; tail -5 $out/${n}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/${n}_$i.json')); print('$n run $i', d['ms_per_step'], d['call_ms_each_step'])"
  done
done
