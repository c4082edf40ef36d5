set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tf_v7 -o run -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_tf_v7.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rnn_v4 -o run -- python bench.py --model RNNModel --mode hyper --attackers 7:Opt-Fang:2 --steps 3 --warmup 1 > gpurun_out/prof_rnn_v4.log 2>&1
