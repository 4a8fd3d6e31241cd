#!/bin/bash
# runtime trace (HIP API + kernels + copies) of the stalled-step pattern
set -u
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-rt}
mkdir -p $out
timeout -k 10 400 rocprofv3 --runtime-trace --output-format csv -d $out/prof -o run -- python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/b.json 2> $out/b.err || { echo rc=$?; tail -5 $out/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/b.json')); print('rt', d['ms_per_step'], d['call_ms_each_step'])"
ls -la $out/prof/*
