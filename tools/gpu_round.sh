# GPU sweep used during development: full GPU suite + bench lines for every config
mkdir -p gpurun_out
timeout -k 10 800 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t_gpu6.log 2>&1; rc=$?
tail -4 gpurun_out/t_gpu6.log
[ $rc -ne 0 ] && exit $rc
run() { F110QP_LANE_MODE=$3 timeout -k 10 200 python bench.py --no-cpu --config $1 --backend $2 > gpurun_out/b_$1_$2_$3.json 2>gpurun_out/b_$1_$2_$3.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/b_$1_$2_$3.json'));print('$1 $2 mode$3', '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), d['config']['mean_active_set_iters'], d['config']['max_active_set_iters'], 'lat1 %.1f'%d['latency']['single_qp_device']['p50_us'])"; }
run c2 wave 0; run c2 lane 0
run c2_big lane 0; run c2_big lane 2
run c4 lane 0
run c5 lane 0; run c5 wave 0; run c5_cold lane 0
run c3 auto 0
