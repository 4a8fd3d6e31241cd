#!/bin/bash
# round 6: Fermat inverse by an addition chain (127 squarings + 12 products): parity tests, the
# host-phase trace of a headline proof (ZKL_HOST_TRACE), and a per-dispatch kernel trace
set -u
out=gpurun_out/r06j
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "headline or deep or ood or fri or lde" > $out/pytest.log 2>&1 || { echo "tests rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
ZKL_HOST_TRACE=1 timeout -k 10 180 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 --programs none > $out/ht.json 2> $out/ht.err || { echo "ht rc=$?"; tail -5 $out/ht.err; exit 1; }
grep "\[ht\]" $out/ht.err | tail -24
bash scripts/gpu_r06g.sh
