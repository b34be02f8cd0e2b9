# lane kernel: predicated HBM scratch writes — parity subset, timing and FETCH/WRITE at c4/c2_big
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "lane or c4 or warm or non_finite or agree or closed" > gpurun_out/l5_tests.log 2>&1 || { tail -30 gpurun_out/l5_tests.log; exit 3; }
tail -1 gpurun_out/l5_tests.log
for c in c4 c2_big; do
timeout -k 10 200 python bench.py --no-cpu --no-latency --config $c --steps 20 > gpurun_out/l5_$c.json 2>/dev/null || exit 9
python -c "import json;d=json.load(open('gpurun_out/l5_$c.json'));print('$c', '%.3e'%d['value'], d['roofline']['kernel_ms_per_launch']*1e3)"
PROF_NAME=l5_$c bash tools/profile_round.sh $c > /dev/null || exit 4
done
