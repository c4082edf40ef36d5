set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_transformer.py tests/test_gpu_chunked.py > gpurun_out/tf_tests.log 2>&1; tail -1 gpurun_out/tf_tests.log
echo "== TF: A tree (laggards' v unit from A) vs B prev"; bash tools/ab_native.sh attackfl_amd/_C_prev.so 3 --steps 20 --warmup 3 || exit 1
