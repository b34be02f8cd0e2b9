# C3: box PDAS first, then GI from its active set for the violated gap rows
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/c3_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/c3_tests.log | head -20; exit 3; }
tail -1 gpurun_out/c3_tests.log
for c in c3 c2; do
timeout -k 10 200 python bench.py --no-cpu --no-latency --config $c --steps 20 > gpurun_out/c3_$c.json 2>/dev/null || exit 9
python -c "import json;d=json.load(open('gpurun_out/c3_$c.json'));c=d['config'];print('$c', '%.3e'%d['value'], '%.1f'%(d['ms_per_step']*1e3), 'k %.1f'%(d['roofline']['kernel_ms_per_launch']*1e3), c['mean_active_set_iters'], c['max_active_set_iters'], c.get('halfspace_kernel_ms'))"
done
