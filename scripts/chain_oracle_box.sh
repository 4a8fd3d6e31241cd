#!/bin/bash
# Oracle proofs of chain segments [start, stop) on the GPU box's host CPUs (no GPU use): the
# 64-segment configs[3] goldens (tests/golden/make_chain_goldens.py), cached under
# gpurun_out/chain_cache and merged back into the build container.
#   bash scripts/chain_oracle_box.sh START STOP THREADS
set -u
mkdir -p gpurun_out/chain_cache
make -s -C oracle
ZKL_CHAIN_CACHE=gpurun_out/chain_cache timeout -k 10 1140 python -u tests/golden/make_chain_goldens.py --skip-agg \
  --start $1 --stop $2 --threads $3 2>&1 | tee gpurun_out/chain_cache/log.txt
