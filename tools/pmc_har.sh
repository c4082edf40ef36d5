#!/bin/bash
# PMC counters of the HAR encoder kernels over one bench round (four rocprofv3 --pmc passes, no tracing domains,
# 6 SQ counters each; summarise with tools/pmc_summary.py gpurun_out/pmc_har).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_har
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_har/p$i -o p$i --output-format csv -- \
    python3 $R/bench.py --model TransformerClassifier --data-name HAR --steps 1 --warmup 1 > $R/gpurun_out/pmc_har/run$i.log 2>&1 || exit $?
done
