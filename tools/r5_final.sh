#!/bin/bash
# Final tree: GPU suite + smoke + default bench, PMC after the image padding, kernel traces of TF / RNN / CNN
set -o pipefail
bash tools/r5_full_tests.sh || exit $?
bash tools/r5_pmc_after.sh || exit $?
bash tools/r5_rocprof_final.sh || exit $?
