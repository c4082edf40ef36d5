#!/bin/bash
# A batch of GPU-box steps chosen by name (each under its own time limit; the first failure ends the batch).
#   tools/gpu_batch.sh har_tests har_bench cnn2_tests study ...
set -o pipefail
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
for s in "$@"; do
  case $s in
    har_tests) step har_tests 400 $PYT tests/test_gpu_har.py tests/test_gpu_programs.py -k "har or TransformerClassifier or attention" ;;
    har_bench) step har_bench 300 python bench.py --model TransformerClassifier --data-name HAR --steps 3 --warmup 1 ;;
    cnn2_tests) step cnn2_tests 300 $PYT tests/test_gpu_programs.py -k "cnn2 or CNNModel" ;;
    cnn_bench) step cnn_bench 300 python bench.py --model CNNModel --steps 10 --warmup 2 ;;
    rnn_bench) step rnn_bench 300 python bench.py --model RNNModel --steps 20 --warmup 3 ;;
    bench) step bench 300 python bench.py --steps 20 --warmup 3 ;;
    gpu_all) step gpu_all 900 $PYT tests -m gpu ;;
    har_prof) step har_prof 320 bash tools/rocprof_har.sh ;;
    valu) step valu_rates 90 ./tools/valu_rates.bin ;;
    study) step study_g10 600 python tools/attack_study.py --device cuda --out gpurun_out/study_gpu_r4_g10.jsonl --genuine-rate 1.0
           step study_g10f 300 python tools/attack_study.py --device cuda --out gpurun_out/study_gpu_r4_g10_flat.jsonl --genuine-rate 1.0 --distance flat
           step study_seeds 300 python tools/attack_study.py --device cuda --out gpurun_out/study_gpu_r4_seeds.jsonl --cells fedavg:Opt-Fang,trimmed_mean:Opt-Fang,trimmed_mean:Random,hyper:Opt-Fang,fedavg:Random --seeds 7,8,9,10,11 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
