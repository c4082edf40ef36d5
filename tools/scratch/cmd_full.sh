set -e -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
OUT=gpurun_out/bench_configs_v5.jsonl bash tools/bench_configs.sh > gpurun_out/sweep.log 2>&1
