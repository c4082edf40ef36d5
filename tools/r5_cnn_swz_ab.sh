#!/bin/bash
# cnn2 tower rows: 16-byte chunks XOR-swizzled by row bit 2 (CNN2_SWZ=1, B = _C_swz.so) vs the tree (swizzle off)
# and the tree vs the build before the swizzle plumbing (_C_nswz.so)
set -o pipefail
AFL_NATIVE_SO=attackfl_amd/_C_swz.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_programs.py tests/test_gpu_chunked.py -k "cnn or CNN" > gpurun_out/swz_tests.log 2>&1 || { tail -15 gpurun_out/swz_tests.log; exit 1; }
echo "cnn tests (swizzle): $(tail -1 gpurun_out/swz_tests.log)"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_programs.py tests/test_gpu_chunked.py -k "cnn or CNN" > gpurun_out/swz0_tests.log 2>&1 || { tail -15 gpurun_out/swz0_tests.log; exit 1; }
echo "cnn tests (tree): $(tail -1 gpurun_out/swz0_tests.log)"
echo "== CNN: A = tree (swizzle off), B = swizzle on"
bash tools/ab_native.sh attackfl_amd/_C_swz.so 4 --steps 20 --warmup 3 --model CNNModel || exit 1
echo "== CNN: A = tree, B = before the swizzle plumbing"
bash tools/ab_native.sh attackfl_amd/_C_nswz.so 3 --steps 20 --warmup 3 --model CNNModel || exit 1
