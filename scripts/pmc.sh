#!/bin/bash
# HBM traffic per kernel dispatch from rocprofv3 PMC counters, one counter per pass
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).  Run on the GPU box from
# the repo root:  bash scripts/pmc.sh [tag]  ->  gpurun_out/<tag>/pmc_{fetch,write}/...
set -u
tag=${1:-pmc}
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 $root/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/pmc_fetch.json 2> $out/pmc_fetch.err || { echo "fetch pass failed rc=$?"; tail -20 $out/pmc_fetch.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 $root/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/pmc_write.json 2> $out/pmc_write.err || { echo "write pass failed rc=$?"; tail -20 $out/pmc_write.err; exit 1; }
cd $root
python3 scripts/pmc_summary.py $out > $out/pmc_summary.json && cat $out/pmc_summary.json
