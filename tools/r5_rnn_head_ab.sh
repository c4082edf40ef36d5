#!/bin/bash
# rnn2 head images padded to 32 B (B = _C_rh.so) vs the tree (16 B)
set -o pipefail
AFL_NATIVE_SO=attackfl_amd/_C_rh.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rnn.py > gpurun_out/rh_tests.log 2>&1 || { tail -15 gpurun_out/rh_tests.log; exit 1; }
echo "rnn tests (variant): $(tail -1 gpurun_out/rh_tests.log)"
echo "== RNN: A = tree, B = head images padded"
bash tools/ab_native.sh attackfl_amd/_C_rh.so 4 --steps 20 --warmup 3 --model RNNModel || exit 1
