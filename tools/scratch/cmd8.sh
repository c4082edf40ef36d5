set -e -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
timeout -k 10 200 python bench.py --steps 6 --warmup 2 --profile-rounds > gpurun_out/lw_fedavg.log 2>&1
timeout -k 10 200 python bench.py --steps 4 --warmup 2 --profile-rounds --attackers 7:Min-Max:2 > gpurun_out/lw_minmax.log 2>&1
timeout -k 10 200 python bench.py --steps 4 --warmup 2 --profile-rounds --mode hyper --attackers 7:Opt-Fang:2 > gpurun_out/lw_hyperfang.log 2>&1
timeout -k 10 200 python bench.py --steps 4 --warmup 2 --profile-rounds --model RNNModel --mode hyper --attackers 7:Opt-Fang:2 > gpurun_out/lw_rnnhyperfang.log 2>&1
