#!/bin/bash
# cnn2: feature rows (LDF 520 -> 528) and own d1 rows (LDD 136 -> 144) padded to 32 B as well (A) vs the tower-only
# padding (B = _C_cnnb.so)
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_programs.py tests/test_gpu_chunked.py -k "cnn or CNN" > gpurun_out/cnnpad3_tests.log 2>&1 || { tail -15 gpurun_out/cnnpad3_tests.log; exit 1; }
tail -1 gpurun_out/cnnpad3_tests.log
echo "== CNN: A = + feature / d1 rows, B = tower rows only"
bash tools/ab_native.sh attackfl_amd/_C_cnnb.so 4 --steps 20 --warmup 3 --model CNNModel || exit 1
