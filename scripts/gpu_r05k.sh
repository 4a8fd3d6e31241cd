#!/bin/bash
# round 5: the 8-stage DIT pass with limb-weighted twiddles (ZKL_NTT_WL=1: 25 multiply-adds and a
# fold per butterfly instead of a REDC) -- wl1 = var_libs/libzkl_hip_wl1.so (a phase's twiddles
# loaded up front, 242 VGPRs), wl2 = this tree (each stage's twiddles before the stage, 165
# VGPRs), against the REDC form -- parity with wl2, then interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05k
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
echo "== parity with ZKL_NTT_WL=1"
ZKL_NTT_WL=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "lde or headline_proof or split or stage" > $out/parity.log 2>&1 || { echo "parity failed"; tail -40 $out/parity.log; exit 1; }
tail -1 $out/parity.log
for i in 1 2; do
  for v in redc wl1 wl2; do
    unset ZKL_HIP_LIB ZKL_NTT_WL
    [ $v != redc ] && export ZKL_NTT_WL=1
    [ $v = wl1 ] && export ZKL_HIP_LIB=$root/var_libs/libzkl_hip_wl1.so
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
      --host-steps 0 > $out/plain_${v}_$i.json 2> $out/plain_${v}_$i.err || { echo "plain rc=$?"; tail -5 $out/plain_${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/plain_${v}_$i.json')); print('$v', d['value'], d['ms_per_step'], d['parity'].get('status'), 'ntt', d['kernel_ms_per_family_untimed_step']['ntt'], 'lde', d['stage_ms_untimed_step']['trace_lde'])"
  done
done
