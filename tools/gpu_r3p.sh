#!/bin/bash
# hyper-mode round anatomy: kernel trace gaps (TransformerModel hyper; RNNModel hyper + Opt-Fang)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_hyp -o run -- python3 bench.py --steps 20 --warmup 3 --mode hyper > gpurun_out/prof_hyp.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_hypr -o run -- python3 bench.py --steps 20 --warmup 3 --mode hyper --model RNNModel --attackers 6:Opt-Fang:2 > gpurun_out/prof_hypr.log 2>&1 || exit 1
