#!/bin/bash
# round-3: parallel CRC + attackers-in-launch check, then clean-vs-attack bench sweep
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_engine.py > gpurun_out/t_r3b.log 2>&1 || exit 1
for a in "" "--attackers 3:Min-Max:2" "--attackers 3:Min-Sum:2" "--attackers 3:LIE:2:0.74"; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 $a >> gpurun_out/b_r3b.log 2>&1 || exit 1
done
