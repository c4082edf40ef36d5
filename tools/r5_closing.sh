#!/bin/bash
# closing GPU batch on the final tree: GPU suite + smoke + default bench, then the model rows of the sweep
set -o pipefail
bash tools/r5_full_tests.sh || exit $?
OUT=gpurun_out/bench_final_r5.jsonl
: > $OUT
for args in "--model TransformerModel" "--model RNNModel" "--model RNNModel --mode hyper --attackers 7:Opt-Fang:2" "--model CNNModel"; do
  # shellcheck disable=SC2086
  timeout -k 10 300 python bench.py --steps 30 --warmup 2 $args > /tmp/bf.log 2>&1 || exit $?
  tail -1 /tmp/bf.log >> $OUT
  tail -1 /tmp/bf.log | cut -c1-150
done
