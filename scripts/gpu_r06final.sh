#!/bin/bash
# Round-6 end pass in two calls (each within gpurun's limit):
#   bash scripts/gpu_r06final.sh tests  -> full GPU suite + smoke
#   bash scripts/gpu_r06final.sh bench  -> default bench line, rocprofv3 kernel stats of a short
#                                          headline-only bench, SQ counters and FETCH/WRITE traffic
set -u
root=$(pwd)
tag=${ZKL_FINAL_TAG:-r06final}
out=$root/gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu rc=$?"; tail -40 $out/pytest_gpu.log; exit 1; }
  tail -2 $out/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $out/smoke.log; exit 1; }
  tail -1 $out/smoke.log
  exit 0
fi
timeout -k 10 900 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['parity']['status'], d['call_ms_each_step']); print(d['kernel_ms_per_family_untimed_step']); print({k: (d[k] or {}).get('value') for k in ('c3_in_gpu_pipeline','c5_single_segment','real_program','cpu_baseline','host_trace') if k in d}); print({k: v.get('value') for k, v in d.get('programs', {}).items()})"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 $root/bench.py --steps 5 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 --programs none > $out/prof_bench.json 2> $out/prof.err || { echo "rocprof rc=$?"; tail -5 $out/prof.err; exit 1; }
cd $root
python3 tools/ktrace_proof.py $(find $out/prof -name "*kernel_trace.csv" | head -1) > $out/proof_timeline.txt || exit 1
tail -1 $out/proof_timeline.txt
bash scripts/pmc_sq_rows.sh $tag/sq || exit 1
bash scripts/pmc_quick.sh $tag/pmcq || exit 1
echo done
