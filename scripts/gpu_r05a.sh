#!/bin/bash
# round 5, first GPU pass: the new multi-rank stub tests, fib-2pow16 end to end, the bench with the
# program lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_comm_stub.py tests/test_fib_2pow16.py > gpurun_out/r05a/pytest.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/r05a/pytest.log; exit 1; }
tail -5 gpurun_out/r05a/pytest.log
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err || { echo "bench failed"; tail -30 gpurun_out/r05a/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r05a/bench.json')); print(d['value'], d['parity']['status']); print(json.dumps(d.get('programs'), indent=1)[:3000]); print(json.dumps(d.get('host_trace',{}).get('per_proof_allocation'), indent=1)[:2000])"
