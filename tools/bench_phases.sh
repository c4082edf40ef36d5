#!/bin/bash
# Per-phase round timings (bench.py --profile-rounds) for the BASELINE configs on one GPU.
# Output: ${OUT:-gpurun_out/bench_phases}/<name>.log (phase JSON lines on stderr + the bench line).
set -e -o pipefail
OUT=${OUT:-gpurun_out/bench_phases}
mkdir -p "$OUT"
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 2 --profile-rounds "$@" > "$OUT/$name.log" 2>&1
  tail -1 "$OUT/$name.log" | cut -c1-140
}
run tf_fedavg --model TransformerModel
run tf_lie --model TransformerModel --attackers "7:LIE:2:0.74"
run tf_minmax --model TransformerModel --attackers "7:Min-Max:2"
run tf_hyper --model TransformerModel --mode hyper
run tf_hyper_fang --model TransformerModel --mode hyper --attackers "7:Opt-Fang:2"
run rnn_hyper_fang --model RNNModel --mode hyper --attackers "7:Opt-Fang:2"
run cnn --model CNNModel
run har --model TransformerClassifier --data-name HAR
