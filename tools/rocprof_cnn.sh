#!/bin/bash
# rocprofv3 kernel statistics of the CNNModel / ICU bench (5 timed rounds after 2 warmups), summary via
# tools/rocprof_summary.py.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn_r5 -o cnn -- \
  python3 bench.py --model CNNModel --steps 5 --warmup 2 > gpurun_out/prof_cnn_r5.log 2>&1
