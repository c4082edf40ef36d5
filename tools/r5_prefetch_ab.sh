#!/bin/bash
# One-trip input prefetch: tf2 (row index one batch ahead) vs the previous build, and the RNN ceiling of the
# same change (rnn2 without the dependent index load: RNN2_ABL_NOORD, wrong rows, timing only).
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_transformer.py > gpurun_out/pf_tf_tests.log 2>&1 || { tail -5 gpurun_out/pf_tf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tf_tests.log
echo "== TF: A = one-trip prefetch, B = previous build"
bash tools/ab_native.sh attackfl_amd/_C_pre.so 4 --steps 20 --warmup 3 || exit 1
echo "== RNN: A = tree, B = no dependent index load (ceiling)"
bash tools/ab_native.sh attackfl_amd/_C_noord.so 3 --steps 20 --warmup 3 --model RNNModel || exit 1
