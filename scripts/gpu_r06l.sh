#!/bin/bash
# round 6: levels of up to 4096 states on the 48-lane form (tree tops from 4096 nodes, FRI leaves
# and draws of <= 4096 items; abvar/pw4k.so) against the 12-lane form there (abvar/base.so):
# Merkle / FRI / transcript parity on pw4k, then hashbench tree + headline bench A/B
set -u
out=gpurun_out/r06l
mkdir -p $out
ZKL_HIP_LIB=$PWD/abvar/pw4k.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "merkle or headline or fri or coin or transcript" > $out/pytest.log 2>&1 || { echo "tests rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
B="bench.py --steps 8 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 --programs none"
for rep in 1 2 3; do
  for v in abvar/base.so abvar/pw4k.so; do
    n=$(basename $v .so)
    ZKL_HIP_LIB=$PWD/$v timeout -k 10 120 python3 tools/hashbench.py --only tree --reps 10 > $out/hb_${n}_$rep.json 2> $out/hb_${n}_$rep.err || { echo "hb $n rc=$?"; exit 1; }
    ZKL_HIP_LIB=$PWD/$v timeout -k 10 180 python3 $B > $out/b_${n}_$rep.json 2> $out/b_${n}_$rep.err || { echo "bench $n rc=$?"; tail -5 $out/b_${n}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);h=json.load(open(sys.argv[4]));print('bench',sys.argv[2],sys.argv[3],d['value'],d['parity']['status'],'tree_ms',h['tree_ms'],d['kernel_ms_per_family_untimed_step'])" $out/b_${n}_$rep.json $n $rep $out/hb_${n}_$rep.json
  done
done
