mkdir -p gpurun_out/v6
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/v6/gpu_tests.log 2>&1 || { tail -30 gpurun_out/v6/gpu_tests.log; exit 3; }
tail -1 gpurun_out/v6/gpu_tests.log
b() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 30 "$@" > gpurun_out/v6/x_$n.json 2>gpurun_out/v6/x_$n.err || { tail -3 gpurun_out/v6/x_$n.err; exit 5; }
 python -c "import json;d=json.load(open('gpurun_out/v6/x_$n.json'));c=d['config'];print('$n', '%.3e'%d['value'], 'k %.1f us'%(d['roofline']['kernel_ms_per_launch']*1e3), c.get('lane_qps_per_wave'), c.get('lane_segments'), c.get('max_active_set_iters'))"; }
b c5 --config c5
b c5_cold --config c5_cold
b c4_8192 --config c4 --batch 8192
b c4 --config c4
b c2big --config c2_big
b c4_16384 --config c4 --batch 16384
b c2 --config c2
timeout -k 10 200 python tools/seg_probe.py 4096 20 > gpurun_out/v6/probe_c5.txt 2>&1 && grep "per pass" gpurun_out/v6/probe_c5.txt
