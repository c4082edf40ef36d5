#!/bin/bash
# Round 5: row-split TransformerModel trainer (split 5) — numerics, then A/B against split 4 at 8 and 1 clients.
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_transformer.py \
  > gpurun_out/split_tests.log 2>&1 || { tail -40 gpurun_out/split_tests.log; exit 1; }
tail -3 gpurun_out/split_tests.log
OUT=gpurun_out/split_ab.jsonl
: > $OUT
for c in 8 1; do
  for sp in 4 5; do
    AFL_TF_SPLIT=$sp timeout -k 10 300 python bench.py --steps 20 --warmup 3 --clients $c > gpurun_out/split_last.log 2>&1
    echo "{\"split\": $sp, \"res\": $(tail -1 gpurun_out/split_last.log)}" >> $OUT
    tail -1 gpurun_out/split_last.log | cut -c1-150
  done
done
