#!/bin/bash
# round 5: DEEP kernel shapes (points per thread x columns in flight) -- plain bench, the DEEP
# family time of the untimed step, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05p
mkdir -p $out
root=$(pwd)
for i in 1 2; do
  for v in base c8 c2 p1c8; do
    lib=$root/zk-lisp_amd/zkl_hip/libzkl_hip.so
    [ $v != base ] && lib=$root/var_libs/libzkl_hip_deep_$v.so
    ZKL_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
      --host-steps 0 > $out/${v}_$i.json 2> $out/${v}_$i.err || { echo "$v rc=$?"; tail -5 $out/${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/${v}_$i.json')); print('$v', d['value'], d['ms_per_step'], d['parity'].get('status'), 'deep', d['kernel_ms_per_family_untimed_step']['deep'], 'stage', d['stage_ms_untimed_step']['deep'])"
  done
done
