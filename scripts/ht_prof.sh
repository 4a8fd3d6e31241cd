# kernel trace of the host-trace bench line: are the 16 MB chunk uploads blit kernels?
export TMPDIR=/tmp
root=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $root/gpurun_out/htprof -o run --output-format csv -- python3 $root/bench.py --steps 1 --warmup 0 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 3 > $root/gpurun_out/htprof.json 2> $root/gpurun_out/htprof.err || exit 1
echo ok
