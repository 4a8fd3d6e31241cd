#!/bin/bash
# host-resident trace entry point under the library's malloc settings vs glibc defaults
set -u
out=$(pwd)/gpurun_out/${1:-htm}
mkdir -p $out
run() { local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --program-steps 0 --host-steps 8 > $out/$name.json 2> $out/$name.err || { echo "$name rc=$?"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); h=d['host_trace']; print('$name', h['ms_per_proof'], h['fraction_of_resident_rate'], h['two_contexts_in_flight']['fraction_of_resident_rate'], d['call_ms_each_step'])"; }
run warm A=1
for i in 1 2 3; do
  run tuned_$i A=1
  run glibc_$i ZKL_MALLOC_TUNE=0
done
