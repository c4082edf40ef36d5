#!/bin/bash
# hyper early launch without the hidden stream sync (cached device index lists): tests, benches, gap trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_multirank.py > gpurun_out/t_r3r.log 2>&1 || exit 1
for a in "--mode hyper" "--mode hyper --model RNNModel --attackers 6:Opt-Fang:2" "--mode hyper --attackers 3:Opt-Fang:2" "--attackers 3:Min-Max:2" "--attackers 3:Min-Sum:2" ""; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 $a >> gpurun_out/b_r3r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_hyp3 -o run -- python3 bench.py --steps 20 --warmup 3 --mode hyper > gpurun_out/prof_hyp3.log 2>&1 || exit 1
