#!/bin/bash
# Round 5: price the RNN branch row split from below.  Stamped phases of the vitals branch workgroup, waves 0 and 4,
# for the current trainer and for the ABL_HALF ablation build (waves 4-7 skip all per-row / per-tile work, so
# waves 0-3 run alone, one wave per SIMD, with half the dW tiles: a row split without its exchanges).
set -o pipefail
mkdir -p gpurun_out
for so in attackfl_amd/_C.so attackfl_amd/_C_rhalf.so; do
  for wv in 0 4; do
    echo "== $so wave $wv"
    AFL_NATIVE_SO=$so timeout -k 10 120 python tools/phase_profile.py --model RNNModel --block 1 --wave $wv 2>/dev/null | grep -v amdgpu.ids || exit 1
  done
done
