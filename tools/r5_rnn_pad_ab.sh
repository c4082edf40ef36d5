#!/bin/bash
# rnn2 gate images (layer 2 or layer 3) with 32-B row padding (wfrag ds_read_b128 conflict-free, wtfrag 4 -> 2
# extra cycles in the gfx950 bank model); only one layer fits the LDS budget.  Numerics of each variant, then A/B.
set -o pipefail
for v in _C_w2.so _C_w3.so; do
  AFL_NATIVE_SO=attackfl_amd/$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rnn.py > gpurun_out/rnnpad_$v.log 2>&1 || { tail -15 gpurun_out/rnnpad_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/rnnpad_$v.log)"
done
echo "== RNN: A = tree, B = layer-3 padding"
bash tools/ab_native.sh attackfl_amd/_C_w3.so 4 --steps 20 --warmup 3 --model RNNModel || exit 1
echo "== RNN: A = tree, B = layer-2 padding"
bash tools/ab_native.sh attackfl_amd/_C_w2.so 4 --steps 20 --warmup 3 --model RNNModel || exit 1
echo "== RNN: A = tree, B = tree before the stride refactor"
bash tools/ab_native.sh attackfl_amd/_C_pad1.so 2 --steps 20 --warmup 3 --model RNNModel || exit 1
