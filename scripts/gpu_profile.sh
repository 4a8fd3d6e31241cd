#!/bin/bash
# rocprofv3 --kernel-trace --stats of the headline bench (5 timed proofs) and the FETCH_SIZE /
# WRITE_SIZE passes (one counter per run, MI355X_MICROARCH.md) of one proof:
#   bash scripts/gpu_profile.sh [tag] -> gpurun_out/<tag>/{prof,pmc_fetch,pmc_write,pmc_summary.json}
set -u
tag=${1:-prof}
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
B="$root/bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-segments 0 --c5-log-n 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 $root/bench.py --steps 5 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 > $out/prof_bench.json 2> $out/prof.err || { echo "stats rc=$?"; tail -5 $out/prof.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 $B > $out/pmc_fetch.json 2> $out/pmc_fetch.err || { echo "fetch pass rc=$?"; tail -5 $out/pmc_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 $B > $out/pmc_write.json 2> $out/pmc_write.err || { echo "write pass rc=$?"; tail -5 $out/pmc_write.err; exit 1; }
cd $root
python3 scripts/pmc_summary.py $out > $out/pmc_summary.json
echo ok
