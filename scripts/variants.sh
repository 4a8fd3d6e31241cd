#!/bin/bash
# Time the stage kernels of several libzkl_hip variants (tools/build_variant.sh) on the box.
# usage: bash scripts/variants.sh tag name1 name2 ...
set -u
tag=$1; shift
mkdir -p gpurun_out/$tag
for v in "$@"; do
  ZKL_HIP_LIB=zk-lisp_amd/build/var/libzkl_hip_$v.so timeout -k 10 300 python tools/hashbench.py >> gpurun_out/$tag/variants.txt 2>> gpurun_out/$tag/variants.err || { echo "variant $v failed rc=$?"; tail -5 gpurun_out/$tag/variants.err; exit 1; }
done
cat gpurun_out/$tag/variants.txt
