#!/bin/bash
# round 6, second pass: (1) tools/latbench with two independent cube chains per lane (is the
# 48-lane cube issue-bound or dependency-bound?); (2) the matrix-pipe cost of the unreduced-cube
# form: row hash with 6 extra zero-B k-steps per tile (PM_MFMA_PROBE_CFG=6 with
# profiles/r06/mfma_probe/probe_variant.patch applied, 78 MFMAs per round,
# digests unchanged) against the shipped build, hashbench + SQ counters; (3) the caller-Vec
# penalty broken down by phase (bench host_trace.per_proof_allocation, ZKL_UP_DEBUG upload lines)
set -u
out=gpurun_out/r06b
mkdir -p $out
timeout -k 5 180 tools/latbench 200 > $out/lat.txt 2>&1 || { echo "latbench rc=$?"; cat $out/lat.txt; exit 1; }
cat $out/lat.txt | grep part
for rep in 1 2; do
  for v in zk-lisp_amd/zkl_hip/libzkl_hip.so abvar/probe6.so; do
    n=$(basename $(dirname $v))_$(basename $v .so)
    ZKL_HIP_LIB=$PWD/$v timeout -k 10 120 python3 tools/hashbench.py --only rows,comp,tree --reps 5 > $out/hb_${n}_$rep.json 2> $out/hb_${n}_$rep.err || { echo "hashbench $n rc=$?"; tail -5 $out/hb_${n}_$rep.err; exit 1; }
    echo "hb $n $rep $(cat $out/hb_${n}_$rep.json)"
  done
done
bash scripts/pmc_sq_ab.sh r06b/sq abvar/probe6.so || exit 1
python3 -c "
import json
for w in ('base','var'):
    d=json.load(open('gpurun_out/r06b/sq/%s/sq_rows.json'%w)); print(w, {k: d.get(k) for k in ('SQ_INSTS_VALU','SQ_INSTS_MFMA','SQ_INSTS_LDS','SQ_WAIT_INST_ANY','SQ_WAVE_CYCLES','SQ_BUSY_CYCLES')})
"
ZKL_UP_DEBUG=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --program-steps 0 --programs none > $out/host.json 2> $out/host.err || { echo "host bench rc=$?"; tail -20 $out/host.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/host.json')); h=d['host_trace']; print(json.dumps({k:h[k] for k in ('value','ms_per_proof','two_contexts_in_flight')})); print(json.dumps(h['per_proof_allocation'], indent=0)[:3000])"
grep "zkl upload" $out/host.err | tail -12
