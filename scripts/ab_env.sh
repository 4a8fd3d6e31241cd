#!/bin/bash
# A/B of library builds and environment knobs: per variant the matrix-core / headline parity
# tests, then bench lines (10 timed proofs) alternating the variants, 2 repetitions.
#   bash scripts/ab_env.sh tag name=path/lib.so[@VAR=val[,VAR=val]] ...
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
run_env() {  # spec -> "ZKL_HIP_LIB=... VAR=val ..."
  local spec=$1 lib envs
  lib=${spec#*=}; envs=""
  if [[ $lib == *@* ]]; then envs=${lib#*@}; lib=${lib%%@*}; fi
  echo "ZKL_HIP_LIB=$lib ${envs//,/ }"
}
for spec in "$@"; do
  name=${spec%%=*}
  env $(run_env "$spec") timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "matrix_core or permute or headline_proof or row_digest_rule or host_trace or lde" > $out/tests_$name.log 2>&1 || { echo "tests $name failed"; tail -20 $out/tests_$name.log; exit 1; }
  echo "$name: $(tail -1 $out/tests_$name.log)"
done
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}
    env $(run_env "$spec") timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 > $out/bench_${name}_$rep.json 2> $out/bench_$name.err || { echo "bench $name failed"; tail -5 $out/bench_$name.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/bench_${name}_$rep.json')); k=d['kernel_ms_per_family_untimed_step']; print('$name', d['ms_per_step'], d['parity']['status'], 'rows', d['roofline']['avg_launch_ms'], 'ntt', k['ntt'], 'ce', k['constraint_eval'], 'deep', k['deep'], 'merkle', k['merkle'], 'comp', k['comp_hash_rows'], 'fri', k['fri'])"
  done
done
