# round 2: state of HEAD on the GPU — full -m gpu suite, then grouped / lane timings (one call)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s_tests.log 2>&1 || { tail -40 gpurun_out/s_tests.log; exit 3; }
tail -3 gpurun_out/s_tests.log
b() { f=gpurun_out/s_$(echo "$@" | tr ' -' '__').json
  timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 20 "$@" > $f 2>gpurun_out/s_err.log || exit 9
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];r=d['roofline'];print(sys.argv[2:], '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['backend'][:40], c['mean_active_set_iters'], c['max_active_set_iters'])" $f "$@"; }
b --config c2
b --config c3
b --config c5
b --config c2_big
b --config c4 --batch 8192 --backend wave --grouped on
b --config c4 --batch 8192 --backend lane
b --config c4 --backend wave --grouped on
b --config c4 --backend lane
b --config c4 --batch 16384 --backend wave --grouped on
b --config c4 --batch 16384 --backend lane
