#!/bin/bash
# End-of-round sweep on the final round-5 tree (after the weight-image padding): every configuration and robust
# mode (30 timed rounds), then the client-count cliff sweep.
set -o pipefail
STEPS=30 OUT=gpurun_out/bench_configs_r5b.jsonl bash tools/bench_configs.sh || exit 1
STEPS=10 bash tools/r5_cliff.sh || exit 1
cp gpurun_out/cliff_r5.jsonl gpurun_out/cliff_r5b.jsonl
