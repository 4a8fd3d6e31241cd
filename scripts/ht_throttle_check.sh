cat /sys/fs/cgroup/cpu.stat 2>/dev/null | grep -E "throttled|usage" ; cat /sys/fs/cgroup/cpu.max 2>/dev/null
for v in "t8:" "t4:ZKL_UP_THREADS=4"; do name=${v%%:*}; envs=${v#*:}
env ZKL_UP_DEBUG=1 $envs timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 5 > gpurun_out/thr_$name.json 2> gpurun_out/thr_$name.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/thr_$name.json')); h=d['host_trace']; print('$name', h['ms_per_proof'], h['upload_loop_ms_last_proof'])"
cat /sys/fs/cgroup/cpu.stat 2>/dev/null | grep -E "throttled"
done
