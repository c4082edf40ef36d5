#!/bin/bash
# Round-5 baseline pass: headline bench, the per-rank 8-GPU proxy (--clients 1), RNN / CNN at 8 and 1 clients.
set -e -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r5_base.jsonl
: > $OUT
run() {
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 "$@" > gpurun_out/r5_base_last.log 2>&1
  tail -1 gpurun_out/r5_base_last.log >> $OUT
  tail -1 gpurun_out/r5_base_last.log | cut -c1-200
}
run
run --clients 1
run --model RNNModel
run --model RNNModel --clients 1
run --model CNNModel --steps 10
