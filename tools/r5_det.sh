#!/bin/bash
# Round 5: new numerics tests (HAR per tensor, FLTrust composite, fixed-point column sums), the on-chip trainer
# suites, then A/B of the fixed-point column sums (A) against the round-4 fp64 atomics (B, -DONCHIP_FP64_COLSUM).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_programs.py \
  tests/test_gpu_transformer.py tests/test_gpu_rnn.py tests/test_gpu_chunked.py \
  "tests/test_gpu_engine.py::test_robust_modes_end_to_end" > gpurun_out/det_tests.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/det_tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
bash tools/ab_native.sh attackfl_amd/_C_ab.so 4 --steps 20 --warmup 3 > gpurun_out/ab_fxsum_tf.log 2>&1 || exit 1
bash tools/ab_native.sh attackfl_amd/_C_ab.so 3 --steps 20 --warmup 3 --model RNNModel > gpurun_out/ab_fxsum_rnn.log 2>&1 || exit 1
cat gpurun_out/ab_fxsum_tf.log gpurun_out/ab_fxsum_rnn.log
bash tools/ab_native.sh attackfl_amd/_C_ab.so 2 --steps 3 --warmup 1 --model TransformerClassifier --data-name HAR > gpurun_out/ab_har_lds.log 2>&1 || exit 1
cat gpurun_out/ab_har_lds.log
