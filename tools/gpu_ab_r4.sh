#!/bin/bash
# round-4 A/B batch: CNN conv3 fragments issued after conv1 instead of at the step start
set -o pipefail
AFL_NATIVE_SO=attackfl_amd/_C_w3late.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_programs.py -k "cnn2 or CNNModel" > gpurun_out/cnnt.log 2>&1; rc=$?; tail -1 gpurun_out/cnnt.log; [ $rc -eq 0 ] || exit $rc
for v in _C _C_w3late; do AFL_NATIVE_SO=attackfl_amd/$v.so timeout -k 10 100 python tools/cnn2_phases.py > gpurun_out/cnnph_$v.log 2>&1 || exit 1; echo "== $v"; grep -E "^step|^fwd|f\." gpurun_out/cnnph_$v.log; done
echo "== CNN A/B (A = current, B = conv3 fragments late)"; timeout -k 10 500 bash tools/ab_native.sh attackfl_amd/_C_w3late.so 4 --model CNNModel --steps 20 --warmup 2 || exit 1
