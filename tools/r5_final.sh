#!/bin/bash
# Final tree: GPU suite + smoke + default bench, then PMC after the image padding
set -o pipefail
bash tools/r5_full_tests.sh || exit $?
bash tools/r5_pmc_after.sh || exit $?
