#!/bin/bash
# round 5: socket power and sclk across whole headline proofs (plain bench, 200 steps, rocm-smi
# read-only samples every ~1 s)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05s
mkdir -p $out
timeout -k 10 200 python3 bench.py --steps 300 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --programs none \
  --host-steps 0 > $out/b.json 2> $out/b.err &
pid=$!
for k in $(seq 1 60); do
  sleep 1
  kill -0 $pid 2>/dev/null || break
  (timeout -k 5 10 rocm-smi --showpower --showclocks > $out/s_$k.txt 2>&1 || true)
  echo "sample $k $(grep -i -E 'power \(W\)|sclk' $out/s_$k.txt | tr -s ' ' | sed 's/GPU\[0\]//g' | tr '\n' ' ')"
done
wait $pid; rc=$?
echo "bench rc=$rc"
python3 -c "import json; d=json.load(open('$out/b.json')); print(d['value'], d['ms_per_step'])"
