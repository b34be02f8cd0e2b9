# round 2: grouped-mode parity + timing (one GPU call)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_grouped.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g_tests.log 2>&1 || { tail -30 gpurun_out/g_tests.log; exit 3; }
tail -3 gpurun_out/g_tests.log
b() { timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 20 "$@" > gpurun_out/g_$(echo "$@" | tr ' -' '__').json 2>gpurun_out/g_err.log || exit 9
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2:], '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), c['backend'], c['mean_active_set_iters'], c['max_active_set_iters'])" gpurun_out/g_$(echo "$@" | tr ' -' '__').json "$@"; }
b --config c4 --batch 8192 --backend wave --grouped on
b --config c4 --batch 8192 --backend wave --grouped off
b --config c4 --batch 8192 --backend lane
b --config c4 --batch 16384 --backend wave --grouped on
b --config c4 --batch 32768 --backend wave --grouped on
b --config c4 --backend wave --grouped on
b --config c4 --backend lane
b --config c4 --batch 1920 --horizon 20 --backend wave --grouped on
b --config c4 --batch 8192 --horizon 20 --backend wave --grouped on
b --config c4 --batch 8192 --horizon 20 --backend lane
b --config c4 --batch 16384 --horizon 20 --backend wave --grouped on
b --config c4 --batch 16384 --horizon 20 --backend lane
b --config c4 --batch 65536 --horizon 20 --backend wave --grouped on
b --config c4 --batch 65536 --horizon 20 --backend lane
