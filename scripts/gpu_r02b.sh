#!/bin/bash
# Round-2 GPU pass (after scripts/gpu_tests.sh): default bench line, 2-rank launcher rehearsal on one GPU
# (configs[3] path incl. the aggregation proof on rank 0), rocprofv3 kernel statistics and the
# FETCH_SIZE / WRITE_SIZE passes of the current build.  Usage (repo root on the box):
#   bash scripts/gpu_r02b.sh [tag]     -> gpurun_out/<tag>/
set -u
tag=${1:-r02b}
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
ZKL_BENCH_DEVICE=0 timeout -k 10 900 python bench.py --gpus 2 --steps 3 --warmup 1 --c5-log-n 0 > $out/bench_2rank_1gpu.json 2> $out/bench2.err || { echo "2-rank bench failed rc=$?"; tail -20 $out/bench2.err; exit 1; }
cat $out/bench_2rank_1gpu.json
export TMPDIR=/tmp
cd /tmp
B="$root/bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-segments 0 --c5-log-n 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 $root/bench.py --steps 5 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 > $out/prof_bench.json 2> $out/prof.err || { echo "stats rc=$?"; tail -5 $out/prof.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 $B > $out/pmc_fetch.json 2> $out/pmc_fetch.err || { echo "fetch pass rc=$?"; tail -5 $out/pmc_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 $B > $out/pmc_write.json 2> $out/pmc_write.err || { echo "write pass rc=$?"; tail -5 $out/pmc_write.err; exit 1; }
cd $root
python3 scripts/pmc_summary.py $out > $out/pmc_summary.json
echo ok
