# Wave vs lane back-end crossover sweep behind the AUTO thresholds (include/f110qp.h), plus the -m gpu
# suite first; lines under profiles/r03/seg/crossover.txt. Usage on the GPU box: bash tools/crossover.sh
mkdir -p gpurun_out/v3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/v3/gpu_tests.log 2>&1 || { tail -30 gpurun_out/v3/gpu_tests.log; exit 3; }
tail -1 gpurun_out/v3/gpu_tests.log
b() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 30 "$@" > gpurun_out/v3/x_$n.json 2>gpurun_out/v3/x_$n.err || { tail -3 gpurun_out/v3/x_$n.err; exit 5; }
 python -c "import json;d=json.load(open('gpurun_out/v3/x_$n.json'));c=d['config'];print('$n', '%.3e'%d['value'], 'k %.1f us'%(d['roofline']['kernel_ms_per_launch']*1e3), c.get('lane_qps_per_wave'), c.get('max_active_set_iters'))"; }
for bt in 512 1024 2048 3072; do b c2_${bt}_lane --config c2 --batch $bt --backend lane; b c2_${bt}_wave --config c2 --batch $bt --backend wave; done
for bt in 256 512 768; do b n40_${bt}_lane --config c2 --horizon 40 --batch $bt --backend lane; b n40_${bt}_wave --config c2 --horizon 40 --batch $bt --backend wave; done
for bt in 2048 3072; do b n30_${bt}_lane --config c2 --horizon 30 --batch $bt --backend lane; b n30_${bt}_wave --config c2 --horizon 30 --batch $bt --backend wave; done
b c2big --config c2_big
b c4 --config c4
