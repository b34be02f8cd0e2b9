# FindHalfSpaces tail: parity tests, timing sweep, C3 bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "half or hs or c3 or gap" > gpurun_out/hs2_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/hs2_tests.log | head -20; exit 3; }
tail -1 gpurun_out/hs2_tests.log
timeout -k 10 200 python -u tools/hs_time.py 2>&1 | grep -v amdgpu.ids || exit 4
timeout -k 10 200 python bench.py --no-cpu --no-latency --config c3 --steps 20 > gpurun_out/hs2_c3.json 2>/dev/null || exit 9
python -c "import json;d=json.load(open('gpurun_out/hs2_c3.json'));c=d['config'];print('c3', '%.3e'%d['value'], '%.1f'%(d['ms_per_step']*1e3), 'k %.1f'%(d['roofline']['kernel_ms_per_launch']*1e3), c.get('halfspace_kernel_ms'))"
