#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per run) over one headline proof only:
#   bash scripts/pmc_quick.sh [tag] -> gpurun_out/<tag>/{pmc_fetch,pmc_write,pmc_summary.json}
set -u
tag=${1:-pmcq}
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
B="$root/bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 --programs none"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 $B > $out/pmc_fetch.json 2> $out/pmc_fetch.err || { echo "fetch pass rc=$?"; tail -5 $out/pmc_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 $B > $out/pmc_write.json 2> $out/pmc_write.err || { echo "write pass rc=$?"; tail -5 $out/pmc_write.err; exit 1; }
cd $root
python3 scripts/pmc_summary.py $out > $out/pmc_summary.json
echo ok
