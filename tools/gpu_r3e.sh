#!/bin/bash
# round-3: granule hand-offs in the on-chip RNN trainer; full phase profiles of both on-chip trainers
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rnn.py > gpurun_out/t_r3e.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/phase_profile.py --clients 8 --block -1 > gpurun_out/phase_tf2_r3e.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/phase_profile.py --clients 8 --block -1 --model RNNModel > gpurun_out/phase_rnn2_r3e.txt 2>&1 || exit 1
for a in "--model RNNModel" "--mode hyper --model RNNModel --attackers 6:Opt-Fang:2" "--mode hyper"; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 $a >> gpurun_out/b_r3e.log 2>&1 || exit 1
done
