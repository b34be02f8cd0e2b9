# closing lane evidence after the u-store removal: smoke, lane bench lines, rocprofv3 passes
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 || { cat gpurun_out/r02/smoke.log; exit 4; }
tail -1 gpurun_out/r02/smoke.log
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r02/bench_$n.json 2> gpurun_out/r02/bench_$n.err || { tail -5 gpurun_out/r02/bench_$n.err; exit 9; }
  python -c "import json;d=json.load(open('gpurun_out/r02/bench_$n.json'));c=d['config'];r=d['roofline'];print('$n', '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['backend'][:14], c['mean_active_set_iters'], c['max_active_set_iters'])"; }
b c4 --config c4 --no-cpu
b c4_shard8192 --config c4 --batch 8192 --no-cpu
b c5 --config c5 --no-cpu
b c5_cold --config c5_cold --no-cpu
b c5_straight --config c5_straight --no-cpu
b c2_big --config c2_big --no-cpu
for c in c4 c5 c2_big; do bash tools/profile_round.sh $c || exit 6; done
PROF_NAME=c4_8192 bash tools/profile_round.sh c4 --batch 8192 || exit 7
