#!/bin/bash
# round 6: evaluator variants after the constraint groups: dot products + Horner bit sums (cedot,
# the shipped build), the same without the dot products (cedot0), the groups alone (ce31), and
# branch-free additions (ce31bf); parity tests of the shipped build first
set -u
out=gpurun_out/r06f
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_programs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "headline or program or real or layout or pose or ram" > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu rc=$?"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
B="bench.py --steps 8 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 3 --programs none"
for rep in 1 2 3; do
  for v in abvar/ce31.so abvar/cedot.so abvar/cedot0.so abvar/ce31bf.so; do
    n=$(basename $v .so)
    ZKL_HIP_LIB=$PWD/$v timeout -k 10 180 python3 $B > $out/b_${n}_$rep.json 2> $out/b_${n}_$rep.err || { echo "bench $n rc=$?"; tail -5 $out/b_${n}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);rp=d.get('real_program',{});print('bench',sys.argv[2],sys.argv[3],d['value'],d['parity']['status'],'ce',d['kernel_ms_per_family_untimed_step']['constraint_eval'],'real',rp.get('ms_per_proof'),rp.get('parity'),(rp.get('kernel_ms_per_family_untimed_step') or {}).get('constraint_eval'))" $out/b_${n}_$rep.json $n $rep
  done
done
