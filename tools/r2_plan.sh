# planning-kernel iteration: parity tests, phase stamps, tick bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_plan.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/plan_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/plan_tests.log | head -30; exit 3; }
tail -1 gpurun_out/plan_tests.log
F110QP_LIB=f110-mpc_amd/lib_stamps/libf110qp.so timeout -k 10 200 python -u tools/plan_stamps.py 1024 2>gpurun_out/pst_err.log || { tail -5 gpurun_out/pst_err.log; exit 4; }
timeout -k 10 200 python bench.py --no-cpu --config tick --steps 50 > gpurun_out/plan_tick.json 2>/dev/null || exit 5
python -c "import json;d=json.load(open('gpurun_out/plan_tick.json'));c=d['config'];print('tick', '%.1f us/step'%(d['ms_per_step']*1e3), 'plan %.1f us'%(c['plan_kernel_ms']*1e3))"
