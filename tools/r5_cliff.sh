#!/bin/bash
# Round 5: client-count cliffs — the on-chip trainers in back-to-back launches of clients that fit.
set -e -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/cliff_r5.jsonl
: > $OUT
run() {
  timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 2 "$@" > gpurun_out/cliff_last.log 2>&1
  tail -1 gpurun_out/cliff_last.log >> $OUT
  tail -1 gpurun_out/cliff_last.log | cut -c1-120
}
run --model CNNModel --clients 8
run --model CNNModel --clients 16
run --model TransformerModel --clients 64
run --model TransformerModel --clients 128
run --model RNNModel --clients 64
run --model RNNModel --clients 128
