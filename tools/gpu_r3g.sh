#!/bin/bash
# wave priorities in the on-chip TransformerModel trainer: per-wave phases + A/B against the no-priority build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_transformer.py > gpurun_out/t_r3g.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/phase_profile.py --clients 8 --block 1 --wave -1 > gpurun_out/phase_prio_b1.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/phase_profile.py --clients 8 --block 0 --wave -1 > gpurun_out/phase_prio_b0.txt 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_native.sh attackfl_amd/_C_ab.so 3 --steps 100 --warmup 10 > gpurun_out/ab_prio.log 2>&1 || exit 1
