#!/bin/bash
# Host-trace entry point (zkl_hip_prove_segment, pageable trace) under upload knobs, 2 reps:
#   bash scripts/ab_host_trace.sh tag  -> gpurun_out/<tag>/ht_<variant>_<rep>.{json,err}
set -u
out=gpurun_out/${1:-ht}
mkdir -p $out
for rep in 1 2; do
  for v in "t8:" "t4:ZKL_UP_THREADS=4" "t16:ZKL_UP_THREADS=16" "direct:ZKL_UP_MODE=direct"; do
    name=${v%%:*}; envs=${v#*:}
    env ZKL_UP_DEBUG=1 $envs timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 5 > $out/ht_${name}_$rep.json 2> $out/ht_${name}_$rep.err || { echo "$name failed"; tail -5 $out/ht_${name}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/ht_${name}_$rep.json')); h=d['host_trace']; print('$name', d['ms_per_step'], h['ms_per_proof'], h['upload_loop_ms_last_proof'], h['two_contexts_in_flight']['fraction_of_resident_rate'])"
    grep "zkl upload" $out/ht_${name}_$rep.err | tail -2
  done
done
