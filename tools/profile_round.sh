# rocprofv3 evidence for one config: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (never combined with tracing domains). Usage: tools/profile_round.sh c4
set -o pipefail
c=$1; shift
name=${PROF_NAME:-$c}  # e.g. PROF_NAME=c4_8192 tools/profile_round.sh c4 --batch 8192
out=gpurun_out/prof_$name
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu --no-latency --config $c --steps 50 "$@" > $out/bench_trace.json 2> $out/trace.err || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py --no-cpu --no-latency --config $c --steps 20 "$@" > $out/bench_fetch.json 2> $out/fetch.err || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py --no-cpu --no-latency --config $c --steps 20 "$@" > $out/bench_write.json 2> $out/write.err || exit 5
echo "profiled $name"
