#!/bin/bash
# one barrier less in the branch update (ffn.0 gradient on waves 0-3): tests, per-wave phases, A/B vs prio-only
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_transformer.py tests/test_gpu_rnn.py > gpurun_out/t_r3h.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/phase_profile.py --clients 8 --block 1 --wave -1 > gpurun_out/phase_h_b1.txt 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_native.sh attackfl_amd/_C_ab.so 3 --steps 100 --warmup 10 > gpurun_out/ab_h.log 2>&1 || exit 1
