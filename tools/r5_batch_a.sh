#!/bin/bash
# batch: world-2 headline repeats, then RNN / CNN trainer PMC passes
set -o pipefail
bash tools/r5_mr2.sh || exit $?
bash tools/r5_pmc_models.sh || exit $?
echo batch-done
