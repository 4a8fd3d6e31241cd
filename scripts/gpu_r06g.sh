#!/bin/bash
# round 6: per-dispatch kernel trace of headline proofs on the current build (where the tree
# tops, iNTT passes and idle gaps go)
set -u
out=$PWD/gpurun_out/r06g
mkdir -p $out
export TMPDIR=/tmp
root=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/kt -o run --output-format csv -- python3 $root/bench.py --steps 3 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 --programs none > $out/b.json 2> $out/b.err || { echo "rc=$?"; tail -5 $out/b.err; exit 1; }
cd $root
python3 tools/ktrace_proof.py $(find $out/kt -name "*kernel_trace.csv" | head -1) > $out/proof_timeline.txt
tail -45 $out/proof_timeline.txt
