#!/bin/bash
# CNN eval head on MFMA: numerics test, eval timing, CNN bench; then the headline's kernel trace (round gaps).
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_programs.py -k "cnn2_eval or prefetch" \
  > gpurun_out/evalhead_tests.log 2>&1 || { tail -30 gpurun_out/evalhead_tests.log; exit 1; }
tail -1 gpurun_out/evalhead_tests.log
timeout -k 10 120 python tools/cnn_eval_bench.py 1 8 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --model CNNModel --steps 20 --warmup 3 2>/dev/null | tail -1 | cut -c1-110 || exit 1
done
rm -rf gpurun_out/prof_tf_r5 && bash tools/rocprof_tf.sh && echo traced
