#!/bin/bash
# A/B of the NTT wide-line mode (ZKL_NTT_WIDE=0/1/2): bench line per mode -> gpurun_out/ab_ntt/
set -u
mkdir -p gpurun_out/ab_ntt
for m in 0 1 2 0; do
  ZKL_NTT_WIDE=$m timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 > gpurun_out/ab_ntt/w$m.json 2> gpurun_out/ab_ntt/w$m.err || { echo "mode $m failed"; tail -5 gpurun_out/ab_ntt/w$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_ntt/w$m.json')); print('mode $m', d['ms_per_step'], d['kernel_ms_per_family_untimed_step']['ntt'], d['stage_ms_untimed_step']['trace_lde'])"
done
