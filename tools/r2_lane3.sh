# round 2: lane kernel v3 (L QPs per wave, single-flip fallback, one launch) parity + L sweep
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "lane or c4 or warm or non_finite or agree" > gpurun_out/l3_tests.log 2>&1 || { tail -40 gpurun_out/l3_tests.log; exit 3; }
tail -3 gpurun_out/l3_tests.log
b() { f=gpurun_out/l3_$(echo "$@" | tr ' -=' '___').json
  timeout -k 10 200 env $1 python bench.py --no-cpu --no-latency --steps 20 ${@:2} > $f 2>gpurun_out/l3_err.log || { cat gpurun_out/l3_err.log; exit 9; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];r=d['roofline'];print(sys.argv[2:], '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['backend'][:12], c['mean_active_set_iters'], c['max_active_set_iters'])" $f "$@"; }
for q in 64 16 8 4; do b F110QP_LANE_QPW=$q --config c4 --batch 8192 --backend lane; done
for q in 64 32; do b F110QP_LANE_QPW=$q --config c4 --backend lane; done
for q in 64 16 8 4 2; do b F110QP_LANE_QPW=$q --config c5 --backend lane; done
for q in 64; do b F110QP_LANE_QPW=$q --config c2_big --backend lane; done
for q in 1 2 4; do b F110QP_LANE_QPW=$q --config c2 --backend lane; done
b X=0 --config c4 --batch 8192 --backend lane
b X=0 --config c4 --backend lane
b X=0 --config c5_cold --backend lane
b X=0 --config c4 --batch 16384 --backend lane
b X=0 --config c4 --batch 4096 --backend lane
b X=0 --config c4 --batch 1024 --backend lane
