#!/bin/bash
# alternating slow proofs: host trace with and without the IFMA host permutation
set -u
out=$(pwd)/gpurun_out/${1:-r04d}
mkdir -p $out
for ifma in 1 0; do
  ZKL_HOST_IFMA=$ifma ZKL_HOST_TRACE=1 timeout -k 10 300 python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/ht_$ifma.json 2> $out/ht_$ifma.err || { echo "rc=$?"; tail -5 $out/ht_$ifma.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/ht_$ifma.json')); print('ifma=$ifma', d['ms_per_step'], d['call_ms_each_step'])"
  grep -E "serialised|stage_events|returned" $out/ht_$ifma.err | tail -9
done
