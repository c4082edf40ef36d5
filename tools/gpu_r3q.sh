#!/bin/bash
# early launch in hyper mode (device-decided hypernetwork update): tests, benches, gap trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_multirank.py tests/test_gpu_ops.py > gpurun_out/t_r3q.log 2>&1 || exit 1
for a in "--mode hyper" "--mode hyper --model RNNModel --attackers 6:Opt-Fang:2" "--mode hyper --attackers 3:Opt-Fang:2"; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 $a >> gpurun_out/b_r3q.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_hyp2 -o run -- python3 bench.py --steps 20 --warmup 3 --mode hyper > gpurun_out/prof_hyp2.log 2>&1 || exit 1
timeout -k 10 700 bash tools/ab_native.sh attackfl_amd/_C_ab.so 4 --steps 100 --warmup 10 > gpurun_out/ab_granule.log 2>&1 || exit 1
