#!/bin/bash
# Where the fixed-point column sums cost time: stamped RNN / TF branch phases, current build vs the fp64-atomics
# variant (_C_fp64.so), waves 0 and 4 of the vitals branch workgroup.
set -o pipefail
for so in attackfl_amd/_C.so attackfl_amd/_C_fp64.so; do
  for wv in 0 4; do
    echo "== RNN $so wave $wv"
    AFL_NATIVE_SO=$so timeout -k 10 120 python tools/phase_profile.py --model RNNModel --block 1 --wave $wv 2>/dev/null | grep -v amdgpu.ids || exit 1
    echo "== TF $so wave $wv"
    AFL_NATIVE_SO=$so timeout -k 10 120 python tools/phase_profile.py --block 1 --wave $wv 2>/dev/null | grep -v amdgpu.ids || exit 1
  done
done
