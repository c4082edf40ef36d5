#!/bin/bash
# round-4 A/B batch: CNN backward image loads during the head wait, with the fc1-image wait at the step start
# (one poll) or before conv3; phases, then bench A/B against the previous build, 4 alternations each
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_programs.py -k "cnn2 or CNNModel" > gpurun_out/cnnt.log 2>&1; rc=$?; tail -2 gpurun_out/cnnt.log; [ $rc -eq 0 ] || exit $rc
for v in _C_prev _C _C_onewait; do AFL_NATIVE_SO=attackfl_amd/$v.so timeout -k 10 100 python tools/cnn2_phases.py > gpurun_out/cnnph_$v.log 2>&1 || exit 1; echo "== $v"; grep -E "^step|^bwd|^fwd|W_barrier" gpurun_out/cnnph_$v.log; done
echo "== CNN A/B (A = split wait, B = previous build)"; timeout -k 10 500 bash tools/ab_native.sh attackfl_amd/_C_prev.so 4 --model CNNModel --steps 20 --warmup 2 || exit 1
echo "== CNN A/B (A = split wait, B = one wait)"; timeout -k 10 500 bash tools/ab_native.sh attackfl_amd/_C_onewait.so 4 --model CNNModel --steps 20 --warmup 2 || exit 1
