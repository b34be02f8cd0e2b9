mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/asm_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/asm_tests.log | head -20; exit 3; }
tail -1 gpurun_out/asm_tests.log
