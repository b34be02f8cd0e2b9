# One rocprofv3 SQ counter pass (8 SQ slots, no tracing domains) per config: wave cycles, the
# disjoint active / wait split (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~
# WAVE_CYCLES), VALU instructions and their active cycles, LDS instructions and LDS issue stalls.
# Usage (repo root, GPU box): bash tools/sq_pass.sh NAME bench.py-args...   -> gpurun_out/sq_NAME/
set -o pipefail
name=$1; shift
out=gpurun_out/sq_$name
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU \
  SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $out/pmc -o run -- \
  python3 bench.py --no-cpu --no-latency --steps 10 --warmup 2 "$@" > $out/bench.json 2> $out/err.log || exit 3
echo "sq pass $name done"
