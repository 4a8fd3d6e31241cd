#!/bin/bash
# Block order of the NTT register pass (ZKL_NTT8_MAP=0/1/2): LDE tests and the headline goldens
# under map 1, then bench lines per map -> gpurun_out/ab_ntt8map/
set -u
out=gpurun_out/ab_ntt8map
mkdir -p $out
ZKL_NTT8_MAP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "lde or ntt or headline_proof_matches_golden" > $out/tests.log 2>&1 || { echo "tests failed"; tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  for m in 0 1 2; do
    ZKL_NTT8_MAP=$m timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 > $out/m${m}_$rep.json 2> $out/m$m.err || { echo "map $m failed"; tail -5 $out/m$m.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/m${m}_$rep.json')); print('map $m', d['ms_per_step'], d['parity']['status'], d['kernel_ms_per_family_untimed_step']['ntt'], d['stage_ms_untimed_step']['trace_lde'])"
  done
done
