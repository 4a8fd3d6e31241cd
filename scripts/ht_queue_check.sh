# host-trace uploads with the default 4 and with 8 HW queues per process
for q in 4 8; do
GPU_MAX_HW_QUEUES=$q ZKL_UP_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --c3-segments 0 --c5-log-n 0 --host-steps 5 > gpurun_out/hq_$q.json 2> gpurun_out/hq_$q.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/hq_$q.json')); h=d['host_trace']; print('queues $q', h['ms_per_proof'], h['upload_loop_ms_last_proof'])"
grep "zkl upload" gpurun_out/hq_$q.err | sed -E 's/.*loop ([0-9.]+) ms \(host copy ([0-9.]+) ms.*waits ([0-9.]+) ms.*/\1\/\3/' | head -6 | tr '\n' ' '; echo
done
