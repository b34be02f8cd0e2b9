# solve-kernel variants (tools/build_solve_variant.sh) against the in-tree library, kernel us
mkdir -p gpurun_out/var
b() { v=$1; shift; lib=f110-mpc_amd/lib/libf110qp.so; [ "$v" != base ] && lib=f110-mpc_amd/lib_var/$v/libf110qp.so
  f=gpurun_out/var/${v}_$(echo "$@" | tr ' -=' '___').json
  F110QP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 50 "$@" > $f 2>gpurun_out/var/err.log || { cat gpurun_out/var/err.log; exit 9; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];c=d['config'];print(sys.argv[2:], 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['solved_fraction'])" $f $v "$@"; }
for v in ${VARS:-base swpe1 swpe2 base}; do
b $v --config c2
b $v --config c3
done
