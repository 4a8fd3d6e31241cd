#!/bin/bash
# NTT register pass A/B, then the row-hash variants (see ab_ntt8.sh, ab_rows.sh)
set -u
bash scripts/ab_ntt8.sh || exit 1
bash scripts/ab_rows.sh zk-lisp_amd/build/var/libzkl_hip_w8.so zk-lisp_amd/build/var/libzkl_hip_w12.so
