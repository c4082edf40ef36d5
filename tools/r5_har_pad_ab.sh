#!/bin/bash
# HAR encoder weight images padded by 32 B (post / post-backward / q|k|v kernels), A = tree vs B = previous build.
set -o pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_har.py tests/test_gpu_programs.py -k "har or HAR" > gpurun_out/harpad_tests.log 2>&1 || { tail -15 gpurun_out/harpad_tests.log; exit 1; }
echo "har tests: $(tail -1 gpurun_out/harpad_tests.log)"
echo "== HAR: A = tree (padded images), B = previous build"
bash tools/ab_native.sh attackfl_amd/_C_pad1.so 3 --model TransformerClassifier --data-name HAR --steps 4 --warmup 1 || exit 1
