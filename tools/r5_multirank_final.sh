#!/bin/bash
# multi-rank regression on the final round-5 tree (N ranks sharing one GPU)
set -o pipefail
OUT=gpurun_out/multirank_r5_final.jsonl bash tools/multirank_sweep.sh 20 5 || exit 1
