#!/bin/bash
# CNNModel step kernel statistics after the deterministic reductions
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnn3 -o cnn -- python3 bench.py --model CNNModel --steps 2 --warmup 1 > gpurun_out/prof_cnn3.log 2>&1 || exit 1
