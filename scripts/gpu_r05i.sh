#!/bin/bash
# round 5: row hashing on the 16-state matrix-core form (ZKL_ROWS_PM16=1) -- parity of the row
# hash stage tests and the headline proof with it, then hashbench rows/comp A/B, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05i
mkdir -p $out
export TMPDIR=/tmp
echo "== parity with ZKL_ROWS_PM16=1"
ZKL_ROWS_PM16=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "hash_rows or headline_proof" > $out/parity.log 2>&1 || { echo "parity failed"; tail -40 $out/parity.log; exit 1; }
tail -1 $out/parity.log
for i in 1 2; do
  for v in pm32 pm16; do
    if [ $v = pm16 ]; then export ZKL_ROWS_PM16=1; else unset ZKL_ROWS_PM16; fi
    timeout -k 10 200 python3 tools/hashbench.py --reps 5 --only rows,comp > $out/hb_${v}_$i.json 2> $out/hb_${v}_$i.err || { echo "hashbench rc=$?"; tail -5 $out/hb_${v}_$i.err; exit 1; }
    echo "$v $i $(cat $out/hb_${v}_$i.json)"
  done
done
unset ZKL_ROWS_PM16
for v in pm32 pm16; do
  if [ $v = pm16 ]; then export ZKL_ROWS_PM16=1; else unset ZKL_ROWS_PM16; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
    --host-steps 0 > $out/plain_$v.json 2> $out/plain_$v.err || { echo "plain rc=$?"; tail -5 $out/plain_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/plain_$v.json')); print('$v', d['value'], d['ms_per_step'], d['parity'].get('status'), d['kernel_ms_per_family_untimed_step'])"
done
