#!/bin/bash
# Per-phase stamps of the final round-5 tree (after the image padding): TF head + vitals branch waves 0 / 4,
# RNN head + vitals branch waves 0 / 4 (tools/phase_profile.py; stamped builds rnn2_stamps / tf2_stamps)
set -o pipefail
mkdir -p gpurun_out
for wv in 0 4; do
  timeout -k 10 120 python tools/phase_profile.py --block 1 --wave $wv 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/phases_tf2_r5_final.txt || exit 1
  timeout -k 10 120 python tools/phase_profile.py --model RNNModel --block 1 --wave $wv 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/phases_rnn2_r5_final.txt || exit 1
done
timeout -k 10 120 python tools/phase_profile.py --block 0 --wave 0 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/phases_tf2_r5_final.txt || exit 1
timeout -k 10 120 python tools/phase_profile.py --model RNNModel --block 0 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/phases_rnn2_r5_final.txt || exit 1
echo phases-done
