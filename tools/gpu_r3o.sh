#!/bin/bash
# early launch at world > 1 (gathered rows): multi-rank tests + multi-rank sweep on one GPU
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_engine.py > gpurun_out/t_r3o.log 2>&1 || exit 1
OUT=gpurun_out/multirank_r3o.jsonl timeout -k 10 900 bash tools/multirank_sweep.sh 60 10 > gpurun_out/multirank_r3o.log 2>&1 || exit 1
