# Same-box A/B of the wave kernel against a variant library (F110QP_LIB): -m gpu on the in-tree
# library, then C2 / C3 / tick kernel times from both. Usage on the GPU box: bash tools/ab_solve_variant.sh
mkdir -p gpurun_out/ab1
V=f110-mpc_amd/lib_var/base/libf110qp.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab1/gpu_tests_var.log 2>&1 || { tail -30 gpurun_out/ab1/gpu_tests_var.log; exit 3; }
tail -1 gpurun_out/ab1/gpu_tests_var.log
for rep in 1 2; do
for lib in f110-mpc_amd/lib/libf110qp.so $V; do
 for c in c2 c3 tick; do
  F110QP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 50 --config $c > gpurun_out/ab1/x.json 2>/dev/null || exit 5
  python -c "import json;d=json.load(open('gpurun_out/ab1/x.json'));print('$lib'.split('/')[-2], '$c', 'k %.2f us'%(d['roofline']['kernel_ms_per_launch']*1e3), d['config']['max_active_set_iters'])"
 done
done
done
for c in "c5" "c4 --batch 8192"; do
  timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 50 --config $c > gpurun_out/ab1/x.json 2>/dev/null || exit 6
  python -c "import json;d=json.load(open('gpurun_out/ab1/x.json'));print('main', '$c', 'k %.2f us'%(d['roofline']['kernel_ms_per_launch']*1e3), d['config']['max_active_set_iters'])"
done
