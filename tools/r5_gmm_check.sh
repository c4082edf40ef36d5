#!/bin/bash
# gmm robust mode: test ROC-AUC of the current tree vs the round-4 kernels (same Python), 10 rounds each.
set -o pipefail
for so in _C _C_r4; do
  echo "== $so"
  AFL_NATIVE_SO=attackfl_amd/$so.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --mode gmm --attackers "7:Min-Max:2" 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['test_roc_auc'], d['rounds_ok'])" || exit 1
  AFL_NATIVE_SO=attackfl_amd/$so.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --mode fltracer --attackers "7:Min-Max:2" 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fltracer', d['value'], d['test_roc_auc'], d['rounds_ok'])" || exit 1
done
