set -u
mkdir -p gpurun_out/ab1
for v in top7 greedy8 w12 w12wide; do echo "== $v"; done
timeout -k 10 200 python tools/hashbench.py --only rows,comp,tree,ntt > gpurun_out/ab1/hb_default.txt 2>&1 || exit 1
for v in top7 greedy8 w12 w12wide; do
  ZKL_HIP_LIB=zk-lisp_amd/build/var/libzkl_hip_$v.so timeout -k 10 200 python tools/hashbench.py --only rows,comp,tree,ntt > gpurun_out/ab1/hb_$v.txt 2>&1 || exit 1
done
cat gpurun_out/ab1/hb_*.txt
timeout -k 10 900 bash scripts/ab_bench.sh ab1 zk-lisp_amd/build/var/libzkl_hip_top7.so zk-lisp_amd/build/var/libzkl_hip_greedy8.so zk-lisp_amd/build/var/libzkl_hip_w12.so zk-lisp_amd/build/var/libzkl_hip_w12wide.so
