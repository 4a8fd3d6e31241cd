#!/bin/bash
# Round-end GPU pass: GPU test suite + smoke, the default bench line, rocprofv3 kernel stats of a
# short bench, and a 2-rank rehearsal on the one GPU:  bash scripts/gpu_final.sh tag
set -u
tag=${1:-final}
out=gpurun_out/$tag
mkdir -p $out
bash scripts/gpu_tests.sh $tag || exit 1
timeout -k 10 500 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
root=$PWD
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/prof -o run --output-format csv -- python3 $root/bench.py --steps 5 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 > $root/$out/prof_bench.json 2> $root/$out/prof.err) || { echo "rocprof rc=$?"; tail -5 $out/prof.err; exit 1; }
ZKL_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --c5-log-n 0 --c3-segments 0 --host-steps 0 > $out/bench_2rank.json 2> $out/bench_2rank.err || { echo "2-rank rc=$?"; tail -20 $out/bench_2rank.err; exit 1; }
echo ok
