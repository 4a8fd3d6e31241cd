#!/bin/bash
# round 5, eighth pass: the 16-state matrix-core form for levels of 2^13 .. 2^16 states --
# stage parity first (fast fail), every GPU parity test, then an interleaved A/B against the
# previous commit's library with a kernel trace of each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05h
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
echo "== stage parity"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "permute or merkle or headline_proof_equals" > $out/stage.log 2>&1 || { echo "stage parity failed"; tail -40 $out/stage.log; exit 1; }
tail -1 $out/stage.log
echo "== parity"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_segments.py tests/test_programs.py > $out/parity.log 2>&1 || { echo "parity failed"; tail -60 $out/parity.log; exit 1; }
tail -1 $out/parity.log
for i in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then export ZKL_HIP_LIB=$root/var_libs/libzkl_hip_prev.so; else unset ZKL_HIP_LIB; fi
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/kt_${v}_$i -o run --output-format csv -- \
      python3 $root/bench.py --steps 3 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
      --host-steps 0 > $root/$out/b_${v}_$i.json 2> $root/$out/b_${v}_$i.err) || { echo "rc=$?"; tail -5 $out/b_${v}_$i.err; exit 1; }
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
      --host-steps 0 > $out/plain_${v}_$i.json 2> $out/plain_${v}_$i.err || { echo "plain rc=$?"; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/plain_${v}_$i.json')); print('$v', d['value'], d['ms_per_step'], d['parity'].get('status'), d['kernel_ms_per_family_untimed_step'])"
  done
done
unset ZKL_HIP_LIB
python3 scripts/kt_compare.py $out/kt_prev_1 $out/kt_new_1 $out/kt_prev_2 $out/kt_new_2 > $out/compare.txt
head -24 $out/compare.txt; tail -1 $out/compare.txt
