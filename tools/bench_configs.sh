#!/bin/bash
# Config sweep of bench.py on one GPU (no attack, LIE, Min-Max, Min-Sum, hyper + Opt-Fang,
# plus the other model families).  One JSON line per config -> ${OUT:-gpurun_out/bench_configs.jsonl}.
set -e -o pipefail
OUT=${OUT:-gpurun_out/bench_configs.jsonl}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
run() {
  timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 "$@" > /tmp/bench_cfg.log 2>&1
  tail -1 /tmp/bench_cfg.log >> "$OUT"
  tail -1 /tmp/bench_cfg.log | cut -c1-160
}
if [ "${SET:-all}" = "robust" ] || [ "${SET:-all}" = "all" ]; then
  # robust server modes (reference server.py:286-494, 682-743), each with one Min-Max attacker
  for m in trimmed_mean median krum shieldfl scionfl FLTrust gmm fltracer byzantine; do
    run --model TransformerModel --mode $m --attackers "7:Min-Max:2"
  done
fi
[ "${SET:-all}" = "robust" ] && exit 0
run --model TransformerModel
run --model TransformerModel --attackers "7:LIE:2:0.74"
run --model TransformerModel --attackers "7:Min-Max:2"
run --model TransformerModel --attackers "7:Min-Sum:2"
run --model TransformerModel --mode hyper
run --model TransformerModel --mode hyper --attackers "7:Opt-Fang:2"
run --model RNNModel
run --model RNNModel --mode hyper --attackers "7:Opt-Fang:2"
run --model CNNModel
run --model TransformerClassifier --data-name HAR
