#!/bin/bash
# End-of-round sweep: every BASELINE configuration and robust mode (tools/bench_configs.sh, 30 timed rounds),
# then the client-count cliff sweep (tools/r5_cliff.sh).
set -o pipefail
STEPS=30 OUT=gpurun_out/bench_configs_r5.jsonl bash tools/bench_configs.sh || exit 1
STEPS=10 bash tools/r5_cliff.sh || exit 1
