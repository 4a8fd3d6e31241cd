#!/bin/bash
# Round-3 A/B of variant libraries: headline golden + matrix-core parity tests per library,
# then bench lines (10 timed proofs) alternating the libraries, 2 repetitions.
#   bash scripts/ab_r03.sh tag lib1.so lib2.so ...
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for v in "$@"; do
  t=$(basename $v .so)
  ZKL_HIP_LIB=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "matrix_core or permute or headline_proof_matches_golden or row_digest_rule" > $out/tests_$t.log 2>&1 || { echo "tests $t failed"; tail -20 $out/tests_$t.log; exit 1; }
  echo "$t: $(tail -1 $out/tests_$t.log)"
done
for rep in 1 2; do
  for v in "$@"; do
    t=$(basename $v .so)
    ZKL_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 > $out/bench_${t}_$rep.json 2> $out/bench_$t.err || { echo "bench $t failed"; tail -5 $out/bench_$t.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/bench_${t}_$rep.json')); k=d['kernel_ms_per_family_untimed_step']; print('$t', d['ms_per_step'], d['parity']['status'], 'rows', d['roofline']['avg_launch_ms'], 'merkle', k['merkle'], 'comp', k['comp_hash_rows'], 'fri', k['fri'])"
  done
done
