#!/bin/bash
# round 5: where the 48-lane round's ~1,600 cycles go (tools/latbench part kernels)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05l
mkdir -p $out
timeout -k 5 120 tools/latbench 200 > $out/lat.txt 2>&1 || { echo "latbench rc=$?"; cat $out/lat.txt; exit 1; }
cat $out/lat.txt
