# full GPU suite, then the bench lines touched by the last change
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/full_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/full_tests.log | head -20; exit 3; }
tail -1 gpurun_out/full_tests.log
for c in ${CONFIGS:-c3 c2 tick}; do
timeout -k 10 200 python bench.py --no-cpu --no-latency --config $c --steps 20 > gpurun_out/full_$c.json 2>/dev/null || exit 9
python -c "import json;d=json.load(open('gpurun_out/full_$c.json'));c=d['config'];print('$c', '%.3e'%d['value'], '%.1f'%(d['ms_per_step']*1e3), 'k %.1f'%(d['roofline']['kernel_ms_per_launch']*1e3), c.get('mean_active_set_iters'), c.get('max_active_set_iters'), c.get('halfspace_kernel_ms'), c.get('plan_kernel_ms'))"
done
