#!/bin/bash
# last GPU batch of the round: the cnn2 row-swizzle A/B, then the final-tree suite, PMC and kernel traces
set -o pipefail
bash tools/r5_cnn_swz_ab.sh || exit $?
bash tools/r5_final.sh || exit $?
