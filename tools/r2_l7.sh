mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "lane or c4 or closed or non_finite" > gpurun_out/l7_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/l7_tests.log | head -20; exit 3; }
tail -1 gpurun_out/l7_tests.log
b() { f=gpurun_out/l7_$(echo "$@" | tr ' -=' '___').json
  timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 20 "$@" > $f 2>/dev/null || exit 9
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];r=d['roofline'];print(sys.argv[2:], '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), 'k %.1f us'%(r['kernel_ms_per_launch']*1e3))" $f "$@"; }
b --config c4
b --config c4 --batch 8192
b --config c5
b --config c5_cold
b --config c2_big
b --config c2 --backend lane
