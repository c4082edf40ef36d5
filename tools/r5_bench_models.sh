#!/bin/bash
# bench.py for each model family on one GPU.
set -o pipefail
for args in "--model TransformerModel" "--model RNNModel" "--model CNNModel" \
            "--model TransformerClassifier --data-name HAR --steps 3 --warmup 1"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 $args 2>/dev/null | tail -1 | cut -c1-140 || exit 1
done
