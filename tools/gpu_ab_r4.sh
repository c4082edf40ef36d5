#!/bin/bash
# round-4 A/B batch: CNN fc1-fragment load position variants (phases, then bench A/B against the current build)
set -o pipefail
for v in _C _C_wf1a _C_wf1b; do AFL_NATIVE_SO=attackfl_amd/$v.so timeout -k 10 100 python tools/cnn2_phases.py > gpurun_out/cnnph_$v.log 2>&1 || exit 1; echo "== $v"; grep -E "step|f\.|fwd " gpurun_out/cnnph_$v.log; done
echo "== CNN A/B (A = current, B = wf1 before conv3)"; timeout -k 10 400 bash tools/ab_native.sh attackfl_amd/_C_wf1a.so 3 --model CNNModel --steps 20 --warmup 2 || exit 1
echo "== CNN A/B (A = current, B = wf1 before conv2)"; timeout -k 10 400 bash tools/ab_native.sh attackfl_amd/_C_wf1b.so 3 --model CNNModel --steps 20 --warmup 2 || exit 1
