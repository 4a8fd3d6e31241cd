#!/bin/bash
# per-dispatch kernel trace of one bench step (for latency analysis of small levels)
set -u
out=$PWD/gpurun_out/${1:-ktrace}
mkdir -p $out
export TMPDIR=/tmp
root=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/kt -o run --output-format csv -- python3 $root/bench.py --steps 1 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 > $out/b.json 2> $out/b.err || { echo "rc=$?"; tail -5 $out/b.err; exit 1; }
ls -R $out | head
