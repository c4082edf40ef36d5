#!/bin/bash
# RNNModel A/B on one box: the current tree (A) against (1) the same source with the unquantised fp64 column-sum
# atomics (_C_fp64.so) and (2) the same source with rnn2's layer-1 16x16x16 MFMA + per-lane vector base in gru_fwd
# taken back out (_C_rnnrev.so, built from a copy outside the tree); then TF against _C_fp64.so.
set -o pipefail
echo "== RNN: current vs fp64 column sums"
bash tools/ab_native.sh attackfl_amd/_C_fp64.so 3 --steps 20 --warmup 3 --model RNNModel || exit 1
echo "== RNN: current vs gru_fwd layer-1 change taken out"
bash tools/ab_native.sh attackfl_amd/_C_rnnrev.so 3 --steps 20 --warmup 3 --model RNNModel || exit 1
echo "== TF: current vs fp64 column sums"
bash tools/ab_native.sh attackfl_amd/_C_fp64.so 3 --steps 20 --warmup 3 || exit 1
