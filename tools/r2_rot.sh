# lane kernel heading frame (ROT): lane parity subset, then timings with the frame on / forced off
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "lane or c4 or warm or non_finite or agree or golden" > gpurun_out/rot_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/rot_tests.log | head -30; tail -30 gpurun_out/rot_tests.log; exit 3; }
tail -2 gpurun_out/rot_tests.log
b() { f=gpurun_out/rot_$(echo "$@" | tr ' -=' '___').json
  timeout -k 10 200 env $1 python bench.py --no-cpu --no-latency --steps 30 ${@:2} > $f 2>gpurun_out/rot_err.log || { cat gpurun_out/rot_err.log; exit 9; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];r=d['roofline'];print(sys.argv[2:], '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['backend'][:12], c['mean_active_set_iters'], c['max_active_set_iters'])" $f "$@"; }
for r in 1; do
b F110QP_LANE_ROT=$r --config c4
b F110QP_LANE_ROT=$r --config c4 --batch 8192
b F110QP_LANE_ROT=$r --config c5
b F110QP_LANE_ROT=$r --config c2_big
done
for d in 0; do
b F110QP_LANE_DREF=$d --config c4 --batch 8192
b F110QP_LANE_DREF=$d --config c5
b F110QP_LANE_DREF=$d --config c2_big
done
