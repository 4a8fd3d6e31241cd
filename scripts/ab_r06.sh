#!/bin/bash
# Round-6 A/B: Poseidon stage kernels (tools/hashbench.py) and short headline benches, the
# libraries given on the command line alternated over three repetitions on one box.
#   bash scripts/ab_r06.sh TAG lib1.so lib2.so ...
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 --programs none"
for rep in 1 2 3; do
  for v in "$@"; do
    n=$(basename $v .so)
    ZKL_HIP_LIB=$v timeout -k 10 120 python3 tools/hashbench.py --only rows,comp,tree --reps 5 > $out/hb_${n}_$rep.json 2> $out/hb_${n}_$rep.err || { echo "hashbench $n rc=$?"; tail -5 $out/hb_${n}_$rep.err; exit 1; }
    echo "hb $n $rep $(cat $out/hb_${n}_$rep.json)"
    ZKL_HIP_LIB=$v timeout -k 10 180 python3 $B > $out/b_${n}_$rep.json 2> $out/b_${n}_$rep.err || { echo "bench $n rc=$?"; tail -5 $out/b_${n}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('bench',sys.argv[2],sys.argv[3],d['value'],d['ms_per_step'],d['parity']['status'],d['kernel_ms_per_family_untimed_step'])" $out/b_${n}_$rep.json $n $rep
  done
done
