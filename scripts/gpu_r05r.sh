#!/bin/bash
# round 5: power and clocks while the row hash runs (rocm-smi read-only queries every ~3 s during
# a long hashbench rows run; one idle reading before)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05r
mkdir -p $out
(timeout -k 5 20 rocm-smi --showpower --showclocks --showtemp > $out/idle.txt 2>&1 || true)
timeout -k 10 150 python3 tools/hashbench.py --reps 1500 --only rows > $out/hb.json 2> $out/hb.err &
pid=$!
for k in $(seq 1 20); do
  sleep 3
  kill -0 $pid 2>/dev/null || break
  (timeout -k 5 10 rocm-smi --showpower --showclocks > $out/busy_$k.txt 2>&1 || true)
  echo "sample $k $(grep -i -E 'power \(W\)|sclk' $out/busy_$k.txt | tr -s ' ' | tr '\n' ' ')"
done
wait $pid; rc=$?
echo "hashbench rc=$rc"; cat $out/hb.json
echo "idle: $(grep -i -E 'power \(W\)|sclk' $out/idle.txt | tr -s ' ' | tr '\n' ' ')"
