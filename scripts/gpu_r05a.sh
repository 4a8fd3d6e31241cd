#!/bin/bash
# round 5, first GPU pass: the new multi-rank stub tests, fib-2pow16 end to end, the paired-element
# round variant (parity + interleaved A/B), the bench with the program lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05a
mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1"; }
step pytest-new
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_comm_stub.py tests/test_fib_2pow16.py tests/test_cpp_host_api.py tests/test_gpu_parity.py::test_grinding_host_continuation_matches_oracle > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
step pair-parity
ZKL_HIP_LIB=$(pwd)/var_libs/libzkl_hip_pair.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "permute or headline_proof_matches_golden or hash_rows or merkle" > $out/pair_parity.log 2>&1 || { echo "pair parity failed"; tail -40 $out/pair_parity.log; exit 1; }
tail -2 $out/pair_parity.log
step ab
for i in 1 2; do
  for v in base pair; do
    if [ $v = pair ]; then export ZKL_HIP_LIB=$(pwd)/var_libs/libzkl_hip_pair.so; else unset ZKL_HIP_LIB; fi
    timeout -k 10 200 python3 tools/hashbench.py --reps 5 --only rows,comp,tree > $out/ab_${v}_$i.json 2> $out/ab_${v}_$i.err || { echo "hashbench $v rc=$?"; tail -5 $out/ab_${v}_$i.err; exit 1; }
    echo "$v $i $(cat $out/ab_${v}_$i.json)"
  done
done
unset ZKL_HIP_LIB
step sq
bash scripts/pmc_sq_ab.sh r05a/sq var_libs/libzkl_hip_pair.so || { echo "sq failed"; exit 1; }
step bench
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || tail -20 $out/bench.err; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
python -c "
import json; d=json.load(open('$out/bench.json'))
print(d['value'], d['ms_per_step'], d['parity'].get('status'), d['parity'].get('failed_lines'), d['roofline']['avg_launch_ms'], d.get('process_tuning'))
for k, v in (d.get('programs') or {}).items(): print(k, json.dumps(v)[:900])
print(json.dumps(d.get('host_trace',{}).get('per_proof_allocation'))[:1500])
print('c3', d.get('c3_in_gpu_pipeline',{}).get('value'), 'c5', d.get('c5_single_segment',{}).get('ms_per_proof'), 'real', d.get('real_program',{}).get('ms_per_proof'))
"
