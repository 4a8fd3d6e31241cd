#!/bin/bash
# round 5, seventh pass: the reseed / FRI coin after each tree in the tree's last launch (17 launches
# fewer per proof) -- parity, then interleaved A/B against the previous commit's library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05g
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
echo "== parity"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_segments.py tests/test_cpp_host_api.py tests/test_programs.py > $out/parity.log 2>&1 || { echo "parity failed"; tail -60 $out/parity.log; exit 1; }
tail -1 $out/parity.log
for i in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then export ZKL_HIP_LIB=$root/var_libs/libzkl_hip_prev.so; else unset ZKL_HIP_LIB; fi
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
      > $out/plain_${v}_$i.json 2> $out/plain_${v}_$i.err || { echo "plain rc=$?"; tail -5 $out/plain_${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/plain_${v}_$i.json')); h=d.get('host_trace',{})
print('$v', d['value'], d['ms_per_step'], d['parity'].get('status'), 'ntt', d['kernel_ms_per_family_untimed_step']['ntt'], 'host', h.get('value'), h.get('ms_per_proof'))"
  done
done
