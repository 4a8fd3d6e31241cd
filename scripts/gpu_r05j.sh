#!/bin/bash
# round 5: the 32-state matrix-core kernels other than row hashing (Merkle levels, FRI leaves,
# draws, grinding) in one 12-wave workgroup per CU (3 waves per SIMD, PM_WAVES_CFG=12
# PM_WIDE_CFG=1: var_libs/libzkl_hip_w12.so) against the shipped 4-wave blocks -- interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05j
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
echo "== w12 parity (Merkle / FRI / headline)"
ZKL_HIP_LIB=$root/var_libs/libzkl_hip_w12.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "merkle or headline_proof_equals or fri" > $out/parity.log 2>&1 || { echo "parity failed"; tail -40 $out/parity.log; exit 1; }
tail -1 $out/parity.log
for i in 1 2 3; do
  for v in cur w12; do
    if [ $v = w12 ]; then export ZKL_HIP_LIB=$root/var_libs/libzkl_hip_w12.so; else unset ZKL_HIP_LIB; fi
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
      --host-steps 0 > $out/plain_${v}_$i.json 2> $out/plain_${v}_$i.err || { echo "plain rc=$?"; tail -5 $out/plain_${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/plain_${v}_$i.json')); print('$v', d['value'], d['ms_per_step'], d['parity'].get('status'), d['kernel_ms_per_family_untimed_step'])"
  done
done
unset ZKL_HIP_LIB
