# C3 GI drop by Givens delete: gap parity tests, stamps, C3/C2 bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "gap or c3 or golden or infeas or horizons or warm or c2 or fallback or refine or custom or true_heading" > gpurun_out/c3d_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/c3d_tests.log | head -20; exit 3; }
tail -1 gpurun_out/c3d_tests.log
F110QP_LIB=f110-mpc_amd/lib_stamps/libf110qp.so timeout -k 10 200 python -u tools/stamps.py 4096 20 gap 2>&1 | grep -v amdgpu.ids | tail -4 || exit 4
for c in c3 c2; do
timeout -k 10 200 python bench.py --no-cpu --no-latency --config $c --steps 20 > gpurun_out/c3d_$c.json 2>/dev/null || exit 9
python -c "import json;d=json.load(open('gpurun_out/c3d_$c.json'));c=d['config'];print('$c', '%.3e'%d['value'], '%.1f'%(d['ms_per_step']*1e3), 'k %.1f'%(d['roofline']['kernel_ms_per_launch']*1e3), c['mean_active_set_iters'], c['max_active_set_iters'], c.get('halfspace_kernel_ms'))"
done
