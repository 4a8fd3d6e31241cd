#!/bin/bash
# Round-4 gap analysis: per-dispatch kernel trace of one proof (where the device idles between
# kernels) and the host timestamps of the transcript round trips (ZKL_HOST_TRACE=1).
set -u
root=$(pwd)
out=$root/gpurun_out/${1:-r04b}
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/kt -o run --output-format csv -- python3 $root/bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/b.json 2> $out/b.err || { echo "rc=$?"; tail -5 $out/b.err; exit 1; }
cd $root
ZKL_HOST_TRACE=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/ht.json 2> $out/ht.err || { echo "rc=$?"; tail -5 $out/ht.err; exit 1; }
f=$(find $out/kt -name "*kernel_trace.csv" | head -1)
python3 tools/ktrace_view.py $f --list > $out/timeline.txt
tail -25 $out/timeline.txt
grep "\[ht\]" $out/ht.err | tail -20
