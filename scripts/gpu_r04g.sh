#!/bin/bash
# split Poseidon evaluator parity + the library's malloc settings against glibc defaults
set -u
root=$(pwd)
out=$root/gpurun_out/${1:-r04g}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_programs.py tests/test_hello_zk.py -m gpu -x -q --timeout 300 --timeout-method thread -k "headline or program or sponge or ram or layouts or golden or hello" > $out/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
run() { local name=$1 extra=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 $extra > $out/$name.json 2> $out/$name.err || { echo "$name rc=$?"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); rp=d.get('real_program') or {}; print('$name', d['ms_per_step'], d['call_ms_each_step'], rp.get('ms_per_proof'), rp.get('parity'), rp.get('kernel_ms_per_family_untimed_step'))"; }
run warm "--program-steps 0" A=1
for i in 1 2; do
  run tuned_$i "" A=1
  run glibc_$i "--program-steps 0" ZKL_MALLOC_TUNE=0
done
