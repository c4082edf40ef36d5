#!/bin/bash
# round-boundary anatomy: per-round host timings + kernel trace gaps of the headline bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AFL_BENCH_TIMES=gpurun_out/times_r3i.jsonl timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > gpurun_out/b_r3i.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gap -o run -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/prof_gap.log 2>&1 || exit 1
