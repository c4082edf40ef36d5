set -e -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
OUT=gpurun_out/bench_configs_v6.jsonl bash tools/bench_configs.sh > gpurun_out/sweep.log 2>&1
timeout -k 10 100 python tools/phase_profile.py --clients 8 --block 1 > gpurun_out/phase_profile_v8_vitals.json 2>&1
timeout -k 10 100 python tools/phase_profile.py --clients 8 --block 0 > gpurun_out/phase_profile_v8_head.json 2>&1
