#!/bin/bash
# Round 5, second pass: CNN eval timing (+ ablations), the numerics of the changed kernels (fp32-only fixed point,
# HAR swizzle), A/B of fixed point vs fp64 and of HAR vs round 4, the RNN half-rows ablation.
set -o pipefail
mkdir -p gpurun_out
for so in _C _C_ev1 _C_ev2 _C_ev3; do
  echo "== cnn eval $so"
  AFL_NATIVE_SO=attackfl_amd/$so.so timeout -k 10 120 python tools/cnn_eval_bench.py 1 8 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_transformer.py \
  tests/test_gpu_rnn.py tests/test_gpu_programs.py -k "transformer or rnn or har or flash or fxsum or determin or split or Transformer or RNN or eval" \
  > gpurun_out/verify2_tests.log 2>&1
rc=$?
grep -E "passed|failed|Error" gpurun_out/verify2_tests.log | tail -8
case $rc in 0|1) ;; *) exit $rc ;; esac
trc=$rc
echo "== fixed point (fp32 conversion) vs fp64 column sums (A = fixed point), TransformerModel"
bash tools/ab_native.sh attackfl_amd/_C_fp64.so 3 --steps 20 --warmup 3 || exit 1
echo "== HAR: round 5 vs round 4 (A = round 5)"
bash tools/ab_native.sh attackfl_amd/_C_r4.so 2 --steps 3 --warmup 1 --model TransformerClassifier --data-name HAR || exit 1
echo "== RNN half-rows ablation"
bash tools/r5_rnn_half.sh || exit 1
exit $trc
