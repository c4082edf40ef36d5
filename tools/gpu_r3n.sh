#!/bin/bash
# early launch of the next round (fedavg, one rank) + RNN trainer wave priorities: tests, benches, A/B, gaps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_rnn.py tests/test_gpu_multirank.py > gpurun_out/t_r3n.log 2>&1 || exit 1
for a in "" "" "--attackers 3:Min-Max:2" "--attackers 3:LIE:2:0.74"; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 $a >> gpurun_out/b_r3n.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/phase_profile.py --clients 8 --block 1 --wave -1 --model RNNModel > gpurun_out/phase_rnn_waves.txt 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_native.sh attackfl_amd/_C_ab.so 3 --steps 60 --warmup 10 --mode hyper --model RNNModel --attackers 6:Opt-Fang:2 > gpurun_out/ab_rnnprio.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gap5 -o run -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/prof_gap5.log 2>&1 || exit 1
