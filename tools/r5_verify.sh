#!/bin/bash
# Round 5 verification pass: the changed kernels' GPU tests, then A/B runs on one box (tools/ab_native.sh):
#   fixed-point column sums vs the fp64 atomics (-DONCHIP_FP64_COLSUM), and the round-5 tree vs the round-4 kernels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_programs.py \
  tests/test_gpu_transformer.py tests/test_gpu_rnn.py tests/test_gpu_chunked.py tests/test_gpu_attacks.py \
  "tests/test_gpu_engine.py::test_robust_modes_end_to_end" > gpurun_out/verify_tests.log 2>&1
rc=$?
grep -E "passed|failed|Error|^\{" gpurun_out/verify_tests.log | tail -8
# numerics failures (rc 1) still let the measurements run; a crash, abort or time limit ends the call
case $rc in 0|1) ;; *) exit $rc ;; esac
trc=$rc
echo "== CNN rocprof (fused eval)"
bash tools/rocprof_cnn.sh && tail -2 gpurun_out/prof_cnn_r5.log || exit 1
echo "== fixed-point vs fp64 column sums (A = fixed point), TransformerModel"
bash tools/ab_native.sh attackfl_amd/_C_fp64.so 4 --steps 20 --warmup 3 || exit 1
echo "== round 5 vs round-4 kernels (A = round 5), TransformerModel"
bash tools/ab_native.sh attackfl_amd/_C_r4.so 3 --steps 20 --warmup 3 || exit 1
echo "== RNNModel"
bash tools/ab_native.sh attackfl_amd/_C_r4.so 3 --steps 20 --warmup 3 --model RNNModel || exit 1
echo "== HAR"
bash tools/ab_native.sh attackfl_amd/_C_r4.so 2 --steps 3 --warmup 1 --model TransformerClassifier --data-name HAR || exit 1
echo "== RNN half-rows ablation"
bash tools/r5_rnn_half.sh || exit 1
exit $trc
