set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tf_v6 -o run -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_tf_v6.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_minmax_v2 -o run -- python bench.py --steps 3 --warmup 1 --attackers 7:Min-Max:2 > gpurun_out/prof_minmax_v2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rnn_hyper -o run -- python bench.py --model RNNModel --mode hyper --attackers 7:Opt-Fang:2 --steps 3 --warmup 1 > gpurun_out/prof_rnn_hyper.log 2>&1
