# Same-box A/B of an environment setting: bench.py kernel time per config, alternating runs
# without and with the assignment. Usage (GPU box): bash tools/ab_env.sh "VAR=value" "c3 c2" [reps]
set -o pipefail
kv=$1; cfgs=$2; reps=${3:-2}
mkdir -p gpurun_out/abenv
for r in $(seq $reps); do
  for c in $cfgs; do
    for v in base set; do
      if [ $v = set ]; then envs="$kv"; else envs=""; fi
      env $envs timeout -k 10 120 python bench.py --config $c --no-cpu --no-latency --steps 50 > gpurun_out/abenv/$c.$v.json 2> gpurun_out/abenv/$c.$v.err || exit 5
      python -c "import json;d=json.load(open('gpurun_out/abenv/$c.$v.json'));print('$r $c $v', '%.2f us'%(d['ms_per_step']*1e3), 'k %.2f'%(d['roofline']['kernel_ms_per_launch']*1e3), d['config'].get('solved_fraction'))"
    done
  done
done
