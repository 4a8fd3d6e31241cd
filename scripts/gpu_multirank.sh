#!/bin/bash
# Rehearse the N-rank bench path on a 1-GPU box: both ranks pinned to device 0.
set -u
out=gpurun_out/${1:-mr}
mkdir -p $out
ZKL_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > $out/bench2.json 2> $out/bench2.err || { echo "2-rank bench failed rc=$?"; tail -30 $out/bench2.err; exit 1; }
cat $out/bench2.json
