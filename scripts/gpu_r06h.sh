#!/bin/bash
# round 6: natural -> bit-reversed NTT passes in the lazy Cooley-Tukey form (ntt_ct_lazy_kernel):
# NTT / LDE stage tests and headline goldens, the full GPU suite, A/B against the canonical DIF
# kernel (ZKL_NTT_CT=0, same library), and a per-dispatch kernel trace of headline proofs
set -u
out=gpurun_out/r06h
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "ntt or lde or headline" > $out/pytest_ntt.log 2>&1 || { echo "ntt tests rc=$?"; tail -40 $out/pytest_ntt.log; exit 1; }
tail -1 $out/pytest_ntt.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu rc=$?"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
B="bench.py --steps 8 --warmup 2 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 0 --program-steps 0 --programs none"
for rep in 1 2 3; do
  for ct in 0 1; do
    ZKL_NTT_CT=$ct timeout -k 10 180 python3 $B > $out/b_ct${ct}_$rep.json 2> $out/b_ct${ct}_$rep.err || { echo "bench ct$ct rc=$?"; tail -5 $out/b_ct${ct}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('bench ct',sys.argv[2],sys.argv[3],d['value'],d['parity']['status'],d['kernel_ms_per_family_untimed_step'])" $out/b_ct${ct}_$rep.json $ct $rep
  done
done
bash scripts/gpu_r06g.sh
