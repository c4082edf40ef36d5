#!/bin/bash
# rnn2 with the dW phases' all-ones operand materialised per phase (A) vs the layer-1 change taken out (B).
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_rnn.py > gpurun_out/rnn_tests.log 2>&1
rc=$?; tail -1 gpurun_out/rnn_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
echo "== RNN: tree vs layer-1 change taken out"
bash tools/ab_native.sh attackfl_amd/_C_rnnrev.so 3 --steps 20 --warmup 3 --model RNNModel || exit 1
exit $rc
