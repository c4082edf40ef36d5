set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
grep -i -E "ICACHE|IFETCH|WAIT_INST|INST_LEVEL" gpurun_out/counters.txt > gpurun_out/counters_ic.txt || true
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace --stats -d gpurun_out/pmc_ic -o run -- python3 tools/phase_profile.py --clients 8 --block 0 > gpurun_out/pmc_ic.log 2>&1
