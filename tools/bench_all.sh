# One bench line per BASELINE config (auto back end) + the default run with the CPU baseline.
mkdir -p gpurun_out/bench_all
timeout -k 10 300 python bench.py > gpurun_out/bench_all/default.json 2> gpurun_out/bench_all/default.err || exit 3
for c in c2 c3 c4 c5 c5_cold c2_big; do
  timeout -k 10 200 python bench.py --no-cpu --config $c > gpurun_out/bench_all/$c.json 2> gpurun_out/bench_all/$c.err || exit 4
done
timeout -k 10 200 python bench.py --no-cpu --config c4 --backend wave --steps 10 > gpurun_out/bench_all/c4_wave.json 2> gpurun_out/bench_all/c4_wave.err || exit 5
timeout -k 10 200 python bench.py --no-cpu --config c5 --backend wave > gpurun_out/bench_all/c5_wave.json 2> gpurun_out/bench_all/c5_wave.err || exit 6
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/bench_all/*.json")):
    d = json.load(open(f)); c = d["config"]; l = d.get("latency", {})
    print(f"{os.path.basename(f):16s} {d['value']:.3e} QP/s {d['ms_per_step']*1e3:8.1f} us/step  {c['backend'][:5]} iters {c['mean_active_set_iters']:.2f}/{c['max_active_set_iters']} "
          f"B1-dev p50 {l.get('single_qp_device',{}).get('p50_us',0):.1f} us host {l.get('single_qp_host_pointers',{}).get('p50_us',0):.1f} us  "
          f"cpu {d.get('cpu_baseline',{}).get('value',0):.3e}")
PY
