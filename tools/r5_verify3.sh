#!/bin/bash
# Round 5, third pass: straight-line fixed-point column sums — numerics, A/B against the fp64 atomics (TF, RNN),
# and the RNN half-rows ablation.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_transformer.py \
  tests/test_gpu_rnn.py tests/test_gpu_programs.py -k "transformer or rnn or Transformer or RNN or har or flash or eval or fxsum or determin" > gpurun_out/verify3_tests.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/verify3_tests.log | tail -8
case $rc in 0|1) ;; *) exit $rc ;; esac
trc=$rc
echo "== fixed point vs fp64 column sums (A = fixed point), TransformerModel"
bash tools/ab_native.sh attackfl_amd/_C_fp64.so 4 --steps 20 --warmup 3 || exit 1
echo "== RNNModel"
bash tools/ab_native.sh attackfl_amd/_C_fp64.so 3 --steps 20 --warmup 3 --model RNNModel || exit 1
echo "== RNN half-rows ablation"
bash tools/r5_rnn_half.sh || exit 1
exit $trc
