#!/bin/bash
# rnn2: the dW phases' all-ones bias operand from an opaque SGPR (no spill / reload in the step loop: scratch
# 52 -> 16 bytes, all of it outside the loop) vs the previous build (a 16-byte reload at dW3, a spill at dW2)
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rnn.py > gpurun_out/ones_tests.log 2>&1 || { tail -15 gpurun_out/ones_tests.log; exit 1; }
echo "rnn tests: $(tail -1 gpurun_out/ones_tests.log)"
echo "== RNN: A = SGPR ones, B = previous build"
bash tools/ab_native.sh attackfl_amd/_C_prev.so 4 --steps 20 --warmup 3 --model RNNModel || exit 1
