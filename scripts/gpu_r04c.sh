#!/bin/bash
# Round-4 check after a change: GPU suite, default bench line, kernel timeline + host trace.
# Usage: bash scripts/gpu_r04c.sh [tag] [skip-tests]
set -u
root=$(pwd)
out=$root/gpurun_out/${1:-r04c}
mkdir -p $out
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -60 $out/pytest_gpu.log; exit 1; }
  tail -3 $out/pytest_gpu.log
fi
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -20 $out/bench.err; cat $out/bench.json; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['parity']['status']); print(d['kernel_ms_per_family_untimed_step']); print(d['stage_ms_untimed_step']); print({k: d[k].get('value') for k in ('c3_in_gpu_pipeline','c5_single_segment','real_program','cpu_baseline','host_trace') if k in d})"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/kt -o run --output-format csv -- python3 $root/bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/kt.json 2> $out/kt.err || { echo "rc=$?"; tail -5 $out/kt.err; exit 1; }
cd $root
ZKL_HOST_TRACE=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/ht.json 2> $out/ht.err || { echo "rc=$?"; tail -5 $out/ht.err; exit 1; }
f=$(find $out/kt -name "*kernel_trace.csv" | head -1)
python3 tools/ktrace_view.py $f --list > $out/timeline.txt
grep "\[ht\]" $out/ht.err | tail -16
