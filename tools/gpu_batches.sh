#!/bin/bash
# The GPU measurement batches behind the round-3 profiles/ files, one function each (run one at a time on the
# GPU box: `bash tools/gpu_batches.sh <name>`).  Every GPU step has its own time limit; the first failure ends
# the batch.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }

tests() {  # the whole GPU suite, one process
  t 1500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_gpu.log 2>&1
}
sweep() {  # all BASELINE configurations + the other model families (profiles/bench_configs_r3.jsonl)
  OUT=gpurun_out/bench_configs_r3.jsonl STEPS=60 t 1000 bash tools/bench_configs.sh > gpurun_out/bench_configs_r3.log 2>&1
}
attacks3() {  # three attackers of eight (profiles/bench_configs_r3b.jsonl)
  for a in "" "--attackers 3:Min-Max:2" "--attackers 3:Min-Sum:2" "--attackers 3:LIE:2:0.74" \
           "--mode hyper" "--mode hyper --model RNNModel --attackers 6:Opt-Fang:2"; do
    t 200 python -u bench.py --steps 100 --warmup 10 $a >> gpurun_out/b_attacks3.log 2>&1 || return 1
  done
}
multirank() {  # N ranks sharing the GPU (profiles/multirank_r3*.{md,jsonl})
  OUT=gpurun_out/multirank.jsonl t 900 bash tools/multirank_sweep.sh 60 10 > gpurun_out/multirank.log 2>&1
}
phases() {  # per-wave phase stamps of both on-chip trainers (profiles/phase_profile_*_r3*.txt)
  t 300 python -u tools/phase_profile.py --clients 8 --block -1 --wave -1 > gpurun_out/phase_tf2.txt 2>&1 &&
  t 300 python -u tools/phase_profile.py --clients 8 --block 1 --wave -1 --model RNNModel > gpurun_out/phase_rnn2.txt 2>&1
}
gaps() {  # GPU idle time between two rounds' training kernels (profiles/round_gaps_*_r3.md)
  t 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gap -o run -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/prof_gap.log 2>&1 &&
  t 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_hyp -o run -- python3 bench.py --steps 20 --warmup 3 --mode hyper > gpurun_out/prof_hyp.log 2>&1
}
pmc() {  # PMC counter passes over the headline bench (profiles/pmc_bench_r3.md)
  t 700 bash tools/pmc_bench.sh
}
ab() {  # A/B of two native builds on one box: build the variant first (AFL_BUILD_OUT / AFL_DEV_DEFINES)
  t 700 bash tools/ab_native.sh attackfl_amd/_C_ab.so 3 --steps 100 --warmup 10 "$@" > gpurun_out/ab.log 2>&1
}

"$@"
