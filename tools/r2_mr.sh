# multi-rank HIP shard test, default bench line (c2 + CPU baseline), 2-rank gloo bench lines
mkdir -p gpurun_out/r02
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02/mr_tests.log 2>&1 || { tail -40 gpurun_out/r02/mr_tests.log; exit 3; }
grep -E "passed|PASSED" gpurun_out/r02/mr_tests.log | tail -3
timeout -k 10 300 python bench.py > gpurun_out/r02/bench_default.json 2> gpurun_out/r02/bench_default.err || { tail -5 gpurun_out/r02/bench_default.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/r02/bench_default.json'));print('default', '%.3e'%d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms_per_launch']*1e3)"
for c in c2 c4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --config $c --no-cpu --no-latency --steps 20 > gpurun_out/r02/bench_2rank_gloo_$c.json 2> gpurun_out/r02/bench_2rank_$c.err || { tail -5 gpurun_out/r02/bench_2rank_$c.err; exit 5; }
python -c "import json;d=json.load(open('gpurun_out/r02/bench_2rank_gloo_$c.json'));print('2rank $c', d['n_gpus'], '%.3e'%d['value'], d['ms_per_step']*1e3, d['config']['batch_per_gpu'])"
done
