#!/bin/bash
# round 6: A/B of the pruned permutations (base = round-5 build, p3 = both prunings, p1 = the
# constant round-1 cubes only), then the second pass (gpu_r06b.sh)
set -u
bash scripts/ab_r06.sh r06c/ab abvar/base.so abvar/p3.so abvar/p1.so || exit 1
bash scripts/gpu_r06b.sh
