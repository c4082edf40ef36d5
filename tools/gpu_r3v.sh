#!/bin/bash
# deterministic split-K / conv weight gradients / CNN head sums: numerics + bitwise tests, CNN bench, PMC passes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_programs.py > gpurun_out/t_r3v.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "CNN or native" >> gpurun_out/t_r3v.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model CNNModel --steps 30 --warmup 3 > gpurun_out/b_r3v.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model TransformerClassifier --data-name HAR --steps 4 --warmup 1 >> gpurun_out/b_r3v.log 2>&1 || exit 1
timeout -k 10 700 bash tools/pmc_bench.sh || exit 1
