#!/bin/bash
# hyper server: next client's rows pass fused into the head Adam — numerics, A/B, kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "hyper" > gpurun_out/t_r3s.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "speculative or hyper or engine_rounds" >> gpurun_out/t_r3s.log 2>&1 || exit 1
timeout -k 10 700 bash tools/ab_native.sh attackfl_amd/_C_ab.so 3 --steps 100 --warmup 10 --mode hyper > gpurun_out/ab_hyperfuse.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_hyp4 -o run -- python3 bench.py --steps 20 --warmup 3 --mode hyper > gpurun_out/prof_hyp4.log 2>&1 || exit 1
