#!/bin/bash
# round 5, fifth pass: boundary-table and composition-column LDEs read their coefficients in
# the first DIT pass (no materialised blowup copies); closing stage events before the last wait
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05e
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
echo "== parity"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_programs.py tests/test_segments.py > $out/parity.log 2>&1 || { echo "parity failed"; tail -60 $out/parity.log; exit 1; }
tail -1 $out/parity.log
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export ZKL_HIP_LIB=$root/var_libs/libzkl_hip_base.so; else unset ZKL_HIP_LIB; fi
    echo "== ktrace $v $i"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/kt_${v}_$i -o run --output-format csv -- \
      python3 $root/bench.py --steps 5 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
      --host-steps 0 > $root/$out/b_${v}_$i.json 2> $root/$out/b_${v}_$i.err) || { echo "rc=$?"; tail -5 $out/b_${v}_$i.err; exit 1; }
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
      --host-steps 0 > $out/plain_${v}_$i.json 2> $out/plain_${v}_$i.err || { echo "plain rc=$?"; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/plain_${v}_$i.json')); print('$v', d['value'], d['ms_per_step'], d['parity'].get('status'), d['call_ms_each_step'])"
  done
done
unset ZKL_HIP_LIB
python3 scripts/kt_compare.py $out/kt_base_1 $out/kt_new_1 $out/kt_base_2 $out/kt_new_2 > $out/compare.txt
head -30 $out/compare.txt; tail -1 $out/compare.txt
