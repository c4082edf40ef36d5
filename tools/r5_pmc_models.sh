#!/bin/bash
# PMC counters of the RNNModel and CNNModel on-chip trainers (k_rnn2_train, k_cnn2_train) over a short bench,
# four rocprofv3 --pmc passes per model (no tracing domains); summarise with tools/pmc_summary.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for model in RNNModel CNNModel; do
  mkdir -p $R/gpurun_out/pmc_$model
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA" \
             "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_BRANCH"; do
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_$model/p$i -o p$i --output-format csv -- \
      python3 $R/bench.py --model $model --steps 3 --warmup 1 > $R/gpurun_out/pmc_$model/run$i.log 2>&1 || exit $?
  done
done
