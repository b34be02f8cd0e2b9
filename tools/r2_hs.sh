# half-space kernel parity + C3 with FindHalfSpaces in the step
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "half_space or c3 or gap or golden" > gpurun_out/h_tests.log 2>&1 || { tail -40 gpurun_out/h_tests.log; exit 3; }
tail -2 gpurun_out/h_tests.log
timeout -k 10 200 python bench.py --no-cpu --no-latency --config c3 --steps 20 > gpurun_out/h_c3.json 2>gpurun_out/h_err.log || { cat gpurun_out/h_err.log; exit 9; }
python -c "import json;d=json.load(open('gpurun_out/h_c3.json'));c=d['config'];print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], c['halfspace_kernel_ms'], c['halfspace_roofline'])"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h_prof -o run -- python3 bench.py --no-cpu --no-latency --config c3 --steps 20 > gpurun_out/h_c3_prof.json 2>gpurun_out/h_prof.err || exit 4
cat gpurun_out/h_prof/*/run_kernel_stats.csv 2>/dev/null | cut -c1-200 || find gpurun_out/h_prof -name "*stats*"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "closed_loop" > gpurun_out/h_cl.log 2>&1 || { tail -30 gpurun_out/h_cl.log; exit 5; }
tail -2 gpurun_out/h_cl.log
for c in c5 c5_cold c5_straight; do for be in lane wave; do
timeout -k 10 200 python bench.py --no-cpu --no-latency --config $c --backend $be --steps 30 > gpurun_out/h_$c_$be.json 2>gpurun_out/h_err.log || { cat gpurun_out/h_err.log; exit 9; }
python -c "import json;d=json.load(open('gpurun_out/h_$c_$be.json'));c=d['config'];print('$c $be', '%.3e'%d['value'], '%.1f'%(d['ms_per_step']*1e3), '%.1f'%(d['roofline']['kernel_ms_per_launch']*1e3), c['mean_active_set_iters'], c['max_active_set_iters'], c.get('warm_key_hit_rate'), c['backend'][:10])"
done; done
