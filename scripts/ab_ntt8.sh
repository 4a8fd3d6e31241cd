#!/bin/bash
# NTT register-pass check + A/B (ZKL_NTT8=0/1): LDE/NTT parity tests, headline goldens, then one
# bench line per mode -> gpurun_out/ab_ntt8/
set -u
out=gpurun_out/ab_ntt8
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "lde or ntt or headline_proof_matches_golden or kernel_forms" > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for m in 0 1 0 1; do
  ZKL_NTT8=$m timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 > $out/m$m.json 2> $out/m$m.err || { echo "mode $m failed"; tail -5 $out/m$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/m$m.json')); print('ntt8 $m', d['ms_per_step'], d['parity']['status'], d['kernel_ms_per_family_untimed_step']['ntt'], d['stage_ms_untimed_step']['trace_lde'], d['stage_ms_untimed_step']['constraint_commitment'])"
done
