#!/bin/bash
# Build a variant of libzkl_hip.so with extra kernel flags, for A/B timing on the GPU box.
#   tools/build_variant.sh NAME "-DPG_WAVES=3"   ->  zk-lisp_amd/build/var/libzkl_hip_NAME.so
set -e
name=$1; flags=$2
cd "$(dirname "$0")/../zk-lisp_amd"
make -s
mkdir -p build/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c csrc/kernels.hip -o build/var/kernels_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/var/libzkl_hip_$name.so build/var/kernels_$name.o \
  build/prover.o build/host_hash.o build/air_host.o build/tracegen.o build/step.o build/verifier.o build/agg.o build/comm.o -ldl
echo build/var/libzkl_hip_$name.so
