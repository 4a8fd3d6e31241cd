#!/bin/bash
# A/B of whole proofs: default library vs variant builds (tools/build_variant.sh) or
# environment settings (NAME=VALUE), alternating
#   bash scripts/ab_bench.sh tag var1.so [ZKL_PM_MIN_ITEMS=32768 ...]
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
B="bench.py --steps 8 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0"
for rep in 1 2; do
  timeout -k 10 180 python3 $B > $out/default_$rep.json 2> $out/default_$rep.err || { echo "default rc=$?"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('default',d['value'],d['kernel_ms_per_family_untimed_step'])" $out/default_$rep.json
  for v in "$@"; do
    case $v in
      *.so) n=$(basename $v .so); ( export ZKL_HIP_LIB=$v; timeout -k 10 180 python3 $B > $out/${n}_$rep.json 2> $out/${n}_$rep.err ) ;;
      *) n=$v; ( export "$v"; timeout -k 10 180 python3 $B > $out/${n}_$rep.json 2> $out/${n}_$rep.err ) ;;
    esac || { echo "$n rc=$?"; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['kernel_ms_per_family_untimed_step'])" $out/${n}_$rep.json $n
  done
done
