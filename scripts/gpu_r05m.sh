#!/bin/bash
# round 5: the row hash at three waves per SIMD again (12-wave workgroups, digests in LDS, 168
# VGPRs, 8 spilled dwords outside the round loop) and its 8-wave digests-in-LDS control, against
# the shipped 8-wave form: tools/hashbench.py rows + comp, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05m
mkdir -p $out
root=$(pwd)
for i in 1 2 3; do
  for v in base w12big big8; do
    lib=$root/zk-lisp_amd/zkl_hip/libzkl_hip.so
    [ $v != base ] && lib=$root/var_libs/libzkl_hip_$v.so
    ZKL_HIP_LIB=$lib timeout -k 10 200 python3 tools/hashbench.py --reps 5 --only rows,comp > $out/${v}_$i.json 2> $out/${v}_$i.err || { echo "$v rc=$?"; tail -5 $out/${v}_$i.err; exit 1; }
    echo "$v $i $(cat $out/${v}_$i.json)"
  done
done
