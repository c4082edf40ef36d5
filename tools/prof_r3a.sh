#!/bin/bash
# round-3 profiling batch: A/B of the wait-loop change, HAR kernel stats, Min-Max overlap
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_native.sh attackfl_amd/_C_ab.so 2 --steps 30 --warmup 5 > gpurun_out/ab.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_har -o har -- python3 bench.py --model TransformerClassifier --data-name HAR --steps 1 --warmup 1 > gpurun_out/prof_har.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_minmax -o mm -- python3 bench.py --attackers 3:Min-Max:2 --steps 3 --warmup 2 > gpurun_out/prof_mm.log 2>&1 || exit 1
