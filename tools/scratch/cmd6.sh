set -e -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_hyper.log 2>&1
OUT=gpurun_out/bench_phases2 bash tools/bench_phases.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_minmax -o run -- python bench.py --steps 3 --warmup 1 --attackers 7:Min-Max:2 > gpurun_out/prof_minmax.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fedavg -o run -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_fedavg.log 2>&1
