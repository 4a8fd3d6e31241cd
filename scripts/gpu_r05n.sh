#!/bin/bash
# round 5: issue rates of the 64-bit shifts and 32-bit carry ops next to the multiply forms, at
# 1, 2, 3 and 8 waves per SIMD (tools/madbench.hip)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05n
mkdir -p $out
timeout -k 5 200 tools/madbench > $out/madbench.txt 2>&1 || { echo "madbench rc=$?"; cat $out/madbench.txt; exit 1; }
cat $out/madbench.txt
