#!/bin/bash
# Variant libraries A/B: LDE / NTT / headline-golden tests per variant, then bench lines
# alternating default and variants.   bash scripts/ab_libs.sh tag lib1.so lib2.so ...
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for v in "$@"; do
  t=$(basename $v .so)
  ZKL_HIP_LIB=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "lde or ntt or headline_proof_matches_golden" > $out/tests_$t.log 2>&1 || { echo "tests $t failed"; tail -20 $out/tests_$t.log; exit 1; }
  echo "$t: $(tail -1 $out/tests_$t.log)"
done
for rep in 1 2; do
  for v in zk-lisp_amd/zkl_hip/libzkl_hip.so "$@"; do
    t=$(basename $v .so)
    ZKL_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 > $out/bench_${t}_$rep.json 2> $out/bench_$t.err || { echo "bench $t failed"; tail -5 $out/bench_$t.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/bench_${t}_$rep.json')); print('$t', d['ms_per_step'], d['parity']['status'], d['kernel_ms_per_family_untimed_step']['ntt'], d['stage_ms_untimed_step']['trace_lde'])"
  done
done
