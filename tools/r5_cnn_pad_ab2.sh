#!/bin/bash
# cnn2: tower + head bf16 rows padded by 32 B (A) vs tower only (_C_pad1.so) and vs the previous build.
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_programs.py tests/test_gpu_chunked.py -k "cnn or CNN" > gpurun_out/cnnpad2_tests.log 2>&1 || { tail -15 gpurun_out/cnnpad2_tests.log; exit 1; }
tail -1 gpurun_out/cnnpad2_tests.log
echo "== CNN: A = tower + head padding, B = tower padding only"
bash tools/ab_native.sh attackfl_amd/_C_pad1.so 4 --steps 20 --warmup 3 --model CNNModel || exit 1
echo "== CNN: A = tower + head padding, B = previous build"
bash tools/ab_native.sh attackfl_amd/_C_pre.so 3 --steps 20 --warmup 3 --model CNNModel || exit 1
