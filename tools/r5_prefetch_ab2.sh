#!/bin/bash
# rnn2 one-trip input prefetch (closed-form walk, row index one batch ahead) vs the previous build.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rnn.py > gpurun_out/pf_rnn_tests.log 2>&1 || { tail -5 gpurun_out/pf_rnn_tests.log; exit 1; }
tail -1 gpurun_out/pf_rnn_tests.log
echo "== RNN: A = one-trip prefetch, B = previous build"
bash tools/ab_native.sh attackfl_amd/_C_pre.so 4 --steps 20 --warmup 3 --model RNNModel || exit 1
