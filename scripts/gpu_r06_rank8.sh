#!/bin/bash
# round 6: the driver's 8-GPU bench command shape rehearsed on ONE GPU: bench.py --gpus 8 starts
# 8 ranks (all pinned to device 0 by ZKL_BENCH_DEVICE), the step-proof gathers run through
# zkl_comm_* over the NCCL-ABI shared-memory stub (ZKL_RCCL_LIB; RCCL refuses duplicate devices).
# Only shrink: configs[4] at 2^18 rows per rank (8 x 2^20 would need ~480 GB of HBM on one card).
# -> gpurun_out/r06_rank8/{bench_rank8.json,bench_rank8.err,mem.txt}
set -u
out=gpurun_out/r06_rank8
mkdir -p $out
( while true; do date +%s >> $out/mem.txt; grep -E "MemAvailable|Mlocked|Shmem:" /proc/meminfo >> $out/mem.txt; sleep 10; done ) &
mon=$!
ZKL_BENCH_DEVICE=0 ZKL_RCCL_LIB=$PWD/tests/stub/libnccl_shm_stub.so timeout -k 10 1100 python3 bench.py --gpus 8 --c5-log-n 18 > $out/bench_rank8.json 2> $out/bench_rank8.err
rc=$?
kill $mon
echo "rc=$rc"
tail -c 3000 $out/bench_rank8.json
[ $rc -eq 0 ] || { tail -30 $out/bench_rank8.err; exit 1; }
