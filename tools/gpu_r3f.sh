#!/bin/bash
# per-wave phase profiles of the on-chip TransformerModel trainer (branch and head workgroups)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/phase_profile.py --clients 8 --block 1 --wave -1 > gpurun_out/phase_waves_b1.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/phase_profile.py --clients 8 --block 0 --wave -1 > gpurun_out/phase_waves_b0.txt 2>&1 || exit 1
