#!/bin/bash
# Alternating slow steps: is the process being CFS-throttled (cgroup cpu.max) or is something
# else on the CPU?  cpu.stat before/after two short benches, thread counts, top CPU users.
set -u
out=$(pwd)/gpurun_out/${1:-diag}
mkdir -p $out
cat /sys/fs/cgroup/cpu.max > $out/cpu_max.txt 2>&1
cat /sys/fs/cgroup/cpu.stat > $out/cpu_stat_0.txt 2>&1
ps -eo pid,nlwp,pcpu,comm --sort=-pcpu | head -15 > $out/ps_0.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 > $out/b$i.json 2> $out/b$i.err || { echo "rc=$?"; tail -5 $out/b$i.err; exit 1; }
  cat /sys/fs/cgroup/cpu.stat > $out/cpu_stat_$i.txt 2>&1
  python3 -c "import json; d=json.load(open('$out/b$i.json')); print('run $i', d['ms_per_step'], d['call_ms_each_step'])"
done
grep -E "nr_throttled|throttled_usec|usage_usec" $out/cpu_stat_*.txt
cat $out/cpu_max.txt; cat $out/ps_0.txt
