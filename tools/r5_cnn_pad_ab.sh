#!/bin/bash
# cnn2 tower activation rows padded by 32 B instead of 16 (ds_read_b128 fragment reads conflict-free in the
# gfx950 banking model, tools/dbg/lds_banks.py): numerics tests, then A/B against the previous build.
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_programs.py tests/test_gpu_chunked.py -k "cnn or CNN" > gpurun_out/cnnpad_tests.log 2>&1 || { tail -15 gpurun_out/cnnpad_tests.log; exit 1; }
tail -1 gpurun_out/cnnpad_tests.log
echo "== CNN: A = 32-B padding, B = previous build"
bash tools/ab_native.sh attackfl_amd/_C_pre.so 4 --steps 20 --warmup 3 --model CNNModel || exit 1
