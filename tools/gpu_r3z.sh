#!/bin/bash
# deterministic HAR / RNN-graph step programs (ordered partial sums everywhere): tests + HAR / CNN benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_programs.py > gpurun_out/t_r3z.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_transformer.py tests/test_gpu_rnn.py >> gpurun_out/t_r3z.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model TransformerClassifier --data-name HAR --steps 6 --warmup 1 > gpurun_out/b_r3z.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model CNNModel --steps 30 --warmup 3 >> gpurun_out/b_r3z.log 2>&1 || exit 1
