#!/bin/bash
# rocprofv3 kernel trace of the headline bench (TransformerModel / ICU, 8 clients): round gaps via tools/round_gaps.py.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tf_r5 -o tf -- \
  python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof_tf_r5.log 2>&1
