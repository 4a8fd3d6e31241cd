#!/bin/bash
# Build a variant of libzkl_hip.so with extra kernel flags, for A/B timing on the GPU box.
#   tools/build_variant.sh NAME "-DPG_WAVES=3" [poseidon|kernels|both]
#     ->  zk-lisp_amd/build/var/libzkl_hip_NAME.so
# The flags go to the named translation unit(s) (default: both); the other objects are the
# normal build's.
set -e
name=$1; flags=$2; which=${3:-both}
cd "$(dirname "$0")/../zk-lisp_amd"
make -s
mkdir -p build/var
hip="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC"
k=build/kernels.o; p=build/poseidon.o
if [ "$which" != poseidon ]; then $hip $flags -c csrc/kernels.hip -o build/var/kernels_$name.o; k=build/var/kernels_$name.o; fi
if [ "$which" != kernels ]; then $hip $flags -c csrc/poseidon.hip -o build/var/poseidon_$name.o; p=build/var/poseidon_$name.o; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/var/libzkl_hip_$name.so $k $p \
  build/prover.o build/host_hash.o build/host_poseidon_ifma.o build/air_host.o build/tracegen.o build/step.o \
  build/verifier.o build/agg.o build/comm.o -ldl
echo build/var/libzkl_hip_$name.so
