#!/bin/bash
# round-4 A/B batch: tf2 block-tile Adam moments issued before the branch backward (vs at the update start)
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_transformer.py > gpurun_out/t_tf.log 2>&1; rc=$?; tail -2 gpurun_out/t_tf.log; [ $rc -eq 0 ] || exit $rc
echo "== TF A/B (A = refactor, B = previous build)"; timeout -k 10 500 bash tools/ab_native.sh attackfl_amd/_C_prev.so 3 --steps 30 --warmup 3 || exit 1
echo "== TF A/B (A = refactor, B = moments early)"; timeout -k 10 500 bash tools/ab_native.sh attackfl_amd/_C_momearly.so 4 --steps 30 --warmup 3 || exit 1
