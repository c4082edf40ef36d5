#!/bin/bash
# prepare-ahead launches + staged FedAvg weights + pinned trainer results: engine tests, bench, gaps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_multirank.py > gpurun_out/t_r3m.log 2>&1 || exit 1
for a in "" "" "--attackers 3:Min-Max:2" "--mode hyper --model RNNModel --attackers 6:Opt-Fang:2"; do
  AFL_BENCH_TIMES=gpurun_out/times_r3m.jsonl timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 $a >> gpurun_out/b_r3m.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gap4 -o run -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/prof_gap4.log 2>&1 || exit 1
