#!/bin/bash
# MFMA NTT pass: LDE/NTT parity tests and headline goldens, then bench with and without it.
set -u
out=gpurun_out/${1:-ntt_mfma}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "lde or ntt or headline_proof_matches_golden or stage" > $out/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for rep in 1 2; do
  for m in 1 0; do
    ZKL_NTT_MFMA=$m timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 > $out/bench_m${m}_$rep.json 2> $out/bench_m$m.err || { echo "bench failed"; tail -5 $out/bench_m$m.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/bench_m${m}_$rep.json')); k=d['kernel_ms_per_family_untimed_step']; print('mfma=$m', d['ms_per_step'], d['parity']['status'], 'ntt', k['ntt'], 'lde', d['stage_ms_untimed_step']['trace_lde'])"
  done
done
