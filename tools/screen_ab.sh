# A/B of the gap-row box screen on C3 (F110QP_GAP_SCREEN=0 off), then the GPU suite.
set -o pipefail
mkdir -p gpurun_out/screen
for v in 1 0; do
  F110QP_GAP_SCREEN=$v timeout -k 10 180 python bench.py --config c3 --no-cpu --no-latency --steps 30 > gpurun_out/screen/c3_$v.json 2> gpurun_out/screen/c3_$v.err || { tail -5 gpurun_out/screen/c3_$v.err; exit 5; }
  python -c "import json;d=json.loads(open('gpurun_out/screen/c3_$v.json').read().strip().splitlines()[-1]);c=d['config'];r=d['roofline'];print('screen=$v', '%.1f us'%(d['ms_per_step']*1e3), 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['backend'][:40], d.get('solved_fraction', c.get('solved_fraction')))"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/screen/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/screen/gpu_tests.log; exit $rc
