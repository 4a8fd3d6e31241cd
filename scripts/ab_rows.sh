#!/bin/bash
# Row-hash variants (register-held merge_many digests; PM_WAVES 8 / 12): matrix-core parity
# tests and the headline goldens per variant library, hashbench and a bench line each.
#   bash scripts/ab_rows.sh lib1.so lib2.so ...   -> gpurun_out/ab_rows/
set -u
out=gpurun_out/ab_rows
mkdir -p $out
for v in "$@"; do
  tag=$(basename $v .so)
  ZKL_HIP_LIB=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "matrix_core or permute or headline_proof_matches_golden or row_digest_rule" > $out/tests_$tag.log 2>&1 || { echo "tests $tag failed"; tail -20 $out/tests_$tag.log; exit 1; }
  echo "$tag: $(tail -1 $out/tests_$tag.log)"
done
for rep in 1 2; do
  for v in "$@"; do
    tag=$(basename $v .so)
    echo "$tag $(ZKL_HIP_LIB=$v timeout -k 10 120 python3 tools/hashbench.py --reps 3 --only rows,comp,tree)" || exit 1
  done
done
for v in "$@"; do
  tag=$(basename $v .so)
  ZKL_HIP_LIB=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 > $out/bench_$tag.json 2> $out/bench_$tag.err || { echo "bench $tag failed"; tail -5 $out/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_$tag.json')); print('$tag', d['ms_per_step'], d['parity']['status'], d['kernel_ms_per_family_untimed_step'])"
done
