#!/bin/bash
# round-4 A/B batch: HAR attention elementwise math in packed fp32 pairs (tests, then bench A/B)
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_har.py tests/test_gpu_programs.py -k "har or TransformerClassifier" > gpurun_out/t_har.log 2>&1; rc=$?; tail -2 gpurun_out/t_har.log; [ $rc -eq 0 ] || exit $rc
echo "== HAR A/B (A = packed pairs, B = previous build)"; timeout -k 10 600 bash tools/ab_native.sh attackfl_amd/_C_prev.so 3 --model TransformerClassifier --data-name HAR --steps 3 --warmup 1 || exit 1
