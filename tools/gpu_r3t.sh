#!/bin/bash
# round-3 config sweep (all BASELINE configurations + the other model families), one box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/bench_configs_r3.jsonl STEPS=60 timeout -k 10 1000 bash tools/bench_configs.sh > gpurun_out/bench_configs_r3.log 2>&1 || exit 1
