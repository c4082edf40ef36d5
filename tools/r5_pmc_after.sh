#!/bin/bash
# PMC after the weight-image padding: TF headline (pmc_bench passes), RNN, CNN trainers
set -o pipefail
R=$GRAFT_REPO_ROOT
bash tools/r5_pmc_models.sh || exit $?
mv $R/gpurun_out/pmc_RNNModel $R/gpurun_out/pmc_RNNModel_after && mv $R/gpurun_out/pmc_CNNModel $R/gpurun_out/pmc_CNNModel_after || exit 1
bash tools/pmc_bench.sh || exit $?
echo pmc-done
