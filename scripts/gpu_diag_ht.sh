#!/bin/bash
# host-trace of the slow steps: a warm-up run, then ZKL_HOST_TRACE=1 with 8 steps
set -u
out=$(pwd)/gpurun_out/${1:-diag_ht}
mkdir -p $out
timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/w.json 2> $out/w.err || exit 1
python3 -c "import json; d=json.load(open('$out/w.json')); print('warm', d['ms_per_step'], d['call_ms_each_step'])"
ZKL_HOST_TRACE=1 timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/h.json 2> $out/h.err || exit 1
python3 -c "import json; d=json.load(open('$out/h.json')); print('ht', d['ms_per_step'], d['call_ms_each_step'])"
