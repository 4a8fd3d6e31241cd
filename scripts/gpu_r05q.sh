#!/bin/bash
# round 5: the 8-stage DIT pass with a rotated (unpadded) LDS tile, 4 waves per SIMD
# (NTT8_ROT_CFG=1, var_libs/libzkl_hip_rot.so) against the padded 3-wave form: parity of the LDE
# stage tests and the proofs with the variant, then hashbench ntt and plain bench, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05q
mkdir -p $out
root=$(pwd)
ZKL_HIP_LIB=$root/var_libs/libzkl_hip_rot.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "lde or headline_proof or split or ntt" > $out/parity.log 2>&1 || { echo "parity failed"; tail -30 $out/parity.log; exit 1; }
tail -1 $out/parity.log
for i in 1 2; do
  for v in base rot; do
    lib=$root/zk-lisp_amd/zkl_hip/libzkl_hip.so
    [ $v != base ] && lib=$root/var_libs/libzkl_hip_$v.so
    ZKL_HIP_LIB=$lib timeout -k 10 200 python3 tools/hashbench.py --reps 5 --only ntt > $out/hb_${v}_$i.json 2> $out/hb_${v}_$i.err || { echo "hb $v rc=$?"; tail -5 $out/hb_${v}_$i.err; exit 1; }
    ZKL_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
      --host-steps 0 > $out/plain_${v}_$i.json 2> $out/plain_${v}_$i.err || { echo "plain $v rc=$?"; tail -5 $out/plain_${v}_$i.err; exit 1; }
    python3 -c "
import json; h=json.load(open('$out/hb_${v}_$i.json')); d=json.load(open('$out/plain_${v}_$i.json')); print('$v', 'hb_ntt', h.get('ntt_ms'), 'bench', d['value'], d['ms_per_step'], d['parity'].get('status'), 'ntt', d['kernel_ms_per_family_untimed_step']['ntt'], 'lde', d['stage_ms_untimed_step']['trace_lde'])"
  done
done
