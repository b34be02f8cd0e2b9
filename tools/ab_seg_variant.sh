# same-box A/B of segmented-kernel variants (tools/build_seg_variant.sh) on C5 and the C4 shard
mkdir -p gpurun_out/abs
timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/abs/seg_tests.log 2>&1 || { tail -20 gpurun_out/abs/seg_tests.log; exit 3; }
tail -1 gpurun_out/abs/seg_tests.log
for rep in 1 2; do
for lib in f110-mpc_amd/lib/libf110qp.so $(ls f110-mpc_amd/lib_var/*/libf110qp.so); do
 for c in "c5" "c4 --batch 8192" "c2 --backend lane"; do
  F110QP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 50 --config $c > gpurun_out/abs/x.json 2>/dev/null || exit 5
  python -c "import json;d=json.load(open('gpurun_out/abs/x.json'));print('$lib'.split('/')[-2], '$c', 'k %.2f us'%(d['roofline']['kernel_ms_per_launch']*1e3))"
 done
done
done
