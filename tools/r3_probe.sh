# round-3 probe of the partitioned-horizon lane kernel: its tests, the fixed/per-pass split and
# the C4 shard sizes of the 1/2/4/8-GPU split
mkdir -p gpurun_out/v4
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/v4/gpu_tests.log 2>&1 || { tail -30 gpurun_out/v4/gpu_tests.log; exit 3; }
tail -1 gpurun_out/v4/gpu_tests.log
timeout -k 10 200 python tools/seg_probe.py 4096 20 > gpurun_out/v4/probe_c5.txt 2>&1 || { tail gpurun_out/v4/probe_c5.txt; exit 4; }
cat gpurun_out/v4/probe_c5.txt
timeout -k 10 200 python tools/seg_probe.py 8192 40 > gpurun_out/v4/probe_c4s.txt 2>&1 || { tail gpurun_out/v4/probe_c4s.txt; exit 4; }
cat gpurun_out/v4/probe_c4s.txt
b() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 30 "$@" > gpurun_out/v4/x_$n.json 2>gpurun_out/v4/x_$n.err || { tail -3 gpurun_out/v4/x_$n.err; exit 5; }
 python -c "import json;d=json.load(open('gpurun_out/v4/x_$n.json'));c=d['config'];print('$n', '%.3e'%d['value'], 'k %.1f us'%(d['roofline']['kernel_ms_per_launch']*1e3), c.get('lane_qps_per_wave'), c.get('lane_segments'), c.get('max_active_set_iters'))"; }
b c5 --config c5
b c4_8192 --config c4 --batch 8192
b c4_16384 --config c4 --batch 16384
b c4_32768 --config c4 --batch 32768
b c2 --config c2
