# Same-box A/B of two builds of libf110qp.so (F110QP_LIB): bench.py kernel time per config,
# alternating the two libraries. Usage (GPU box): bash tools/ab_lib.sh PREV_SO "c2 c3 c5" [reps]
set -o pipefail
prev=$1; cfgs=$2; reps=${3:-2}
mkdir -p gpurun_out/ab
for r in $(seq $reps); do
  for c in $cfgs; do
    for lib in cur prev; do
      if [ $lib = prev ]; then export F110QP_LIB=$prev; else unset F110QP_LIB; fi
      timeout -k 10 120 python bench.py --config $c --no-cpu --no-latency --steps 50 > gpurun_out/ab/$c.$lib.json 2> gpurun_out/ab/$c.$lib.err || exit 5
      python -c "import json;d=json.load(open('gpurun_out/ab/$c.$lib.json'));print('$r $c $lib', '%.2f us'%(d['ms_per_step']*1e3), 'k %.2f'%(d['roofline']['kernel_ms_per_launch']*1e3))"
    done
  done
done
