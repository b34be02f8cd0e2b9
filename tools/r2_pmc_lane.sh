# SQ counters of the lane kernel at 1 wave per CU (L=64) vs 1 wave per SIMD (L=8), c4 shard
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcl
for q in 64 8; do
  F110QP_LANE_QPW=$q timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmcl/a$q -o run -- python3 bench.py --no-cpu --no-latency --config c4 --batch 8192 --backend lane --steps 3 --warmup 1 > gpurun_out/pmcl/a$q.json 2> gpurun_out/pmcl/a$q.err || exit 3
  F110QP_LANE_QPW=$q timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmcl/b$q -o run -- python3 bench.py --no-cpu --no-latency --config c4 --batch 8192 --backend lane --steps 3 --warmup 1 > gpurun_out/pmcl/b$q.json 2> gpurun_out/pmcl/b$q.err || exit 4
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmcl/*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "lane_kernel" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[2], {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(acc.items())})
PY
