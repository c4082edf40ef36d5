#!/bin/bash
# CNNModel: on-chip trainer tests, then A/B (A = tree, B = _C_head.so: the committed kernels) and per-phase stamps.
set -o pipefail
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_programs.py -k "cnn" \
  > gpurun_out/cnn_tests.log 2>&1
rc=$?
tail -2 gpurun_out/cnn_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
echo "== CNN A/B (A = tree, B = committed)"
bash tools/ab_native.sh attackfl_amd/_C_head.so 3 --steps 10 --warmup 2 --model CNNModel || exit 1
for so in _C _C_head; do
  echo "== phases $so"
  AFL_NATIVE_SO=attackfl_amd/$so.so timeout -k 10 180 python tools/cnn2_phases.py 2>&1 | grep -v amdgpu.ids | head -40 || exit 1
done
exit $rc
