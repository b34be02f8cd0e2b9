# round 2: lane kernel v2 parity + timing (one GPU call)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/l_tests.log 2>&1 || { tail -40 gpurun_out/l_tests.log; exit 3; }
tail -3 gpurun_out/l_tests.log
b() { f=gpurun_out/l_$(echo "$@" | tr ' -' '__').json
  timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 20 "$@" > $f 2>gpurun_out/l_err.log || exit 9
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2:], '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), c['backend'][:30], c['mean_active_set_iters'], c['max_active_set_iters'])" $f "$@"; }
b --config c4 --batch 8192 --backend lane
b --config c4 --backend lane
b --config c2_big
b --config c5
b --config c5_cold
b --config c2 --backend lane
b --config c4 --batch 16384 --backend lane
b --config c4 --batch 32768 --backend lane
