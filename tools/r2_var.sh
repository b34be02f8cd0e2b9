# lane-kernel variants (tools/build_lane_variant.sh) against the in-tree library, kernel us
mkdir -p gpurun_out/var
b() { v=$1; shift; lib=f110-mpc_amd/lib/libf110qp.so; [ "$v" != base ] && lib=f110-mpc_amd/lib_var/$v/libf110qp.so
  f=gpurun_out/var/${v}_$(echo "$@" | tr ' -=' '___').json
  F110QP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-latency --steps 30 "$@" > $f 2>gpurun_out/var/err.log || { cat gpurun_out/var/err.log; exit 9; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];c=d['config'];print(sys.argv[2:], 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['solved_fraction'])" $f $v "$@"; }
for v in ${VARS:-base newton1 ring1}; do
b $v --config c4 --batch 8192
b $v --config c5
b $v --config c2_big
b $v --config c4
done
