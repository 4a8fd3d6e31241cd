#!/bin/bash
# round 5, fourth pass: the host query plan without allocations (plan into per-context scratch,
# addresses straight into the pinned staging buffer, proof bytes written in place) -- parity,
# host phase timings against var_libs/libzkl_hip_base.so, and a two-rank bench rehearsal on one
# GPU through the NCCL-ABI stub (the RCCL code path of the sharded bench lines)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r05d
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
echo "== parity"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  > $out/parity.log 2>&1 || { echo "parity failed"; tail -60 $out/parity.log; exit 1; }
tail -1 $out/parity.log
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export ZKL_HIP_LIB=$root/var_libs/libzkl_hip_base.so; else unset ZKL_HIP_LIB; fi
    ZKL_HOST_TRACE=1 timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c3-segments 0 \
      --c5-log-n 0 --programs none --host-steps 0 > $out/ht_${v}_$i.json 2> $out/ht_${v}_$i.err || { echo "bench $v rc=$?"; tail -5 $out/ht_${v}_$i.err; exit 1; }
    python3 - $out/ht_${v}_$i.err $out/ht_${v}_$i.json $v <<'PY'
import json, statistics, sys
rows = [l.split() for l in open(sys.argv[1]) if l.startswith("[ht]")]
seq = [(r[1], float(r[2])) for r in rows]
d = {}
for (a, ta), (b, tb) in zip(seq, seq[1:]):
    if tb >= ta:
        d.setdefault(f"{a}->{b}", []).append(tb - ta)
j = json.load(open(sys.argv[2]))
print(sys.argv[3], j["value"], j["ms_per_step"], {k: round(statistics.median(v), 1) for k, v in d.items() if k.startswith(("rem", "q_", "serial", "stage"))})
PY
  done
done
unset ZKL_HIP_LIB
echo "== two ranks on one GPU over the stub"
ZKL_BENCH_DEVICE=0 ZKL_RCCL_LIB=$root/tests/stub/libnccl_shm_stub.so timeout -k 10 900 python3 bench.py --gpus 2 --steps 3 \
  --warmup 1 --no-cpu-baseline --c5-log-n 0 --host-steps 0 > $out/rank2.json 2> $out/rank2.err
rc=$?; echo "rank2 rc=$rc"; [ $rc -eq 0 ] || { tail -30 $out/rank2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/rank2.json'))
print(d['value'], d['ms_per_step'], d['n_gpus'], d['parity'].get('status'), json.dumps(d.get('step_handoff'))[:400])
for k in ('c3_in_gpu_pipeline','c4_sharded'):
    if k in d: print(k, json.dumps(d[k])[:600])
for k, v in (d.get('programs') or {}).items(): print(k, {a: b for a, b in v.items() if not isinstance(b, (list, dict))})
"
