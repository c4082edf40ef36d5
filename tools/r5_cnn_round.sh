#!/bin/bash
# CNN round composition after the validation prefetch: the prefetch test, 3 benches, a kernel trace.
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_programs.py tests/test_gpu_engine.py -k "prefetch or cnn2 or cnn or engine or robust or graph or har" \
  > gpurun_out/cnn_round_tests.log 2>&1 || { tail -20 gpurun_out/cnn_round_tests.log; exit 1; }
tail -1 gpurun_out/cnn_round_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model CNNModel --steps 20 --warmup 3 2>/dev/null | tail -1 | cut -c1-120 || exit 1
done
rm -rf gpurun_out/prof_cnn_r5 && bash tools/rocprof_cnn.sh && echo traced
