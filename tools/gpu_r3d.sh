#!/bin/bash
# round-3: granule hand-offs (tf2) + Gram-form attack spectral norms — correctness, phase profile, benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_transformer.py tests/test_gpu_engine.py > gpurun_out/t_r3d.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/phase_profile.py --clients 8 > gpurun_out/phase_r3d.txt 2>&1 || exit 1
for a in "" "" "--attackers 3:Min-Max:2" "--attackers 3:Min-Sum:2" "--attackers 3:LIE:2:0.74" "--mode hyper --model RNNModel --attackers 6:Opt-Fang:2"; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 $a >> gpurun_out/b_r3d.log 2>&1 || exit 1
done
