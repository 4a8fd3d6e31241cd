#!/bin/bash
# round 6: HBM traffic per kernel after the one-pass OOD kernel (FETCH/WRITE passes over one
# headline proof) and SQ counters per kernel (where the constraint evaluator's time goes)
set -u
bash scripts/pmc_quick.sh r06d/pmcq || exit 1
python3 scripts/pmc_traffic.py gpurun_out/r06d/pmcq/pmc_summary.json > gpurun_out/r06d/pmc_traffic.json || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r06d/pmc_traffic.json'))['per_kernel']
for k in ('constraint_eval_kernel<false>','ood_kernel','deep_kernel','hash_rows_pm_kernel<0, false>','ntt_dit8_kernel'): print(k, d.get(k))"
bash scripts/pmc_sq_proof.sh r06d/sq
