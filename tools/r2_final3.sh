# closing check on the final code: whole -m gpu suite, smoke, then SQ counters of the lane kernel
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r02/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r02/gpu_tests.log | head -20; exit 3; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 || { cat gpurun_out/r02/smoke.log; exit 4; }
tail -1 gpurun_out/r02/smoke.log
bash tools/r2_pmc_lane.sh || exit 5
