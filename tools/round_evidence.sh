# Round evidence on one MI355X (profiles/<round>/): the -m gpu suite, smoke(), one bench line per
# BASELINE config (+ the C4 shard sizes of 2/4/8 GPUs), rocprofv3
# kernel stats + FETCH_SIZE / WRITE_SIZE passes of the dominant kernel (tools/profile_round.sh),
# SQ counter passes (tools/sq_pass.sh) and a 2-rank rehearsal of the multi-process bench.
# Usage (repo root, on the GPU box): bash tools/round_evidence.sh r04 [part]
#   part = tests | bench | prof | all (default all); then on the host:
#   python tools/summarize_profiles.py r04 c2 c3 c4 c5 c2_big c4_8192 c4_16384
#   python tools/summarize_sq.py r04 c2:lane_seg_kernel c4_8192:lane_seg_kernel c4_16384:lane_seg_kernel c3:solve_kernel
set -o pipefail
rnd=${1:-r06}
part=${2:-all}
out=gpurun_out/$rnd
mkdir -p $out
export TMPDIR=/tmp
if [ $part = tests ] || [ $part = all ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 3; }
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 4; }
tail -1 $out/smoke.log
fi
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $out/bench_$n.json 2> $out/bench_$n.err || { tail -5 $out/bench_$n.err; exit 5; }
  python -c "import json;d=json.load(open('$out/bench_$n.json'));c=d['config'];r=d['roofline'];print('$n', '%.3e'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), 'k %.1f us'%(r['kernel_ms_per_launch']*1e3), c['backend'][:12], c.get('lane_segments'), d['dtype'], c['mean_active_set_iters'], c['max_active_set_iters'], 'traffic', r.get('traffic'))"; }
if [ $part = bench ] || [ $part = all ]; then
b default
b c2 --config c2 --no-cpu
b c3 --config c3 --no-cpu
b c4 --config c4 --no-cpu
b c4_shard8192 --config c4 --batch 8192 --no-cpu --no-latency
b c4_shard16384 --config c4 --batch 16384 --no-cpu --no-latency
b c4_shard32768 --config c4 --batch 32768 --no-cpu --no-latency
b c5 --config c5 --no-cpu
b c5_cold --config c5_cold --no-cpu
b c5_straight --config c5_straight --no-cpu
b c2_big --config c2_big --no-cpu
b tick --config tick --no-cpu
fi
if [ $part = prof ] || [ $part = all ]; then
for c in c2 c3 c4 c5 c2_big; do bash tools/profile_round.sh $c || exit 6; done
PROF_NAME=c4_8192 bash tools/profile_round.sh c4 --batch 8192 || exit 7
PROF_NAME=c4_16384 bash tools/profile_round.sh c4 --batch 16384 || exit 7
bash tools/sq_pass.sh c2 --config c2 || exit 9
bash tools/sq_pass.sh c4_8192 --config c4 --batch 8192 || exit 9
bash tools/sq_pass.sh c4_16384 --config c4 --batch 16384 || exit 9
bash tools/sq_pass.sh c3 --config c3 || exit 9
timeout -k 10 300 python tools/c2_growth_probe.py > $out/c2_growth_probe.txt 2>&1 || exit 10
timeout -k 10 300 python tools/recheck_counts.py > $out/recheck_counts.json 2> $out/recheck_counts.err || exit 11
for c in c2 c4; do  # bench.py starts its two ranks itself (gloo: both on GPU 0)
  timeout -k 10 300 python bench.py --gpus 2 --config $c --dist-backend gloo --no-cpu --no-latency --steps 20 \
    2> $out/bench_2rank_$c.err | grep "^{\"metric\"" > $out/bench_2rank_gloo_$c.json || exit 8
done
fi
echo evidence done
