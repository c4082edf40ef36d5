#!/bin/bash
# rocprofv3 kernel statistics of the HAR TransformerClassifier bench (one timed round after one warmup).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_har -o har -- \
  python3 bench.py --model TransformerClassifier --data-name HAR --steps 1 --warmup 1 > gpurun_out/prof_har.log 2>&1
