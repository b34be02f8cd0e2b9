mkdir -p gpurun_out
timeout -k 10 800 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t_gpu10.log 2>&1; rc=$?
tail -3 gpurun_out/t_gpu10.log
[ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 200 python bench.py --no-cpu --no-latency --config $1 --backend $2 --steps 30 > gpurun_out/z_$1_$2.json 2>gpurun_out/z_$1_$2.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/z_$1_$2.json'));print('$1 $2', '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), d['config']['mean_active_set_iters'], d['config']['max_active_set_iters'])"; }
run c2 wave; run c2 lane; run c2_big lane; run c4 lane; run c5 lane; run c5_cold lane; run c5 wave; run c3 wave
