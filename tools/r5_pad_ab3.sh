#!/bin/bash
# Weight-image row padding (gfx950 bank model, tools/dbg/lds_banks.py): rnn2 both gate images padded (tree) and
# tf2 variants (head images hpad, branch v / out_proj images + compact dense image bpad, both bhpad).
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rnn.py > gpurun_out/pad3_rnn_tests.log 2>&1 || { tail -15 gpurun_out/pad3_rnn_tests.log; exit 1; }
echo "rnn tests (tree): $(tail -1 gpurun_out/pad3_rnn_tests.log)"
for v in _C_hpad.so _C_bpad.so _C_bhpad.so; do
  AFL_NATIVE_SO=attackfl_amd/$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_transformer.py > gpurun_out/pad3_tf_$v.log 2>&1 || { tail -15 gpurun_out/pad3_tf_$v.log; exit 1; }
  echo "tf tests ($v): $(tail -1 gpurun_out/pad3_tf_$v.log)"
done
echo "== RNN: A = tree (both gate images padded), B = previous build"
bash tools/ab_native.sh attackfl_amd/_C_pad1.so 4 --steps 20 --warmup 3 --model RNNModel || exit 1
echo "== RNN: A = tree, B = layer 3 only"
bash tools/ab_native.sh attackfl_amd/_C_w3.so 2 --steps 20 --warmup 3 --model RNNModel || exit 1
for v in _C_hpad.so _C_bpad.so _C_bhpad.so; do
  echo "== TF: A = tree, B = $v"
  bash tools/ab_native.sh attackfl_amd/$v 4 --steps 20 --warmup 3 || exit 1
done
