set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_transformer.py tests/test_gpu_chunked.py > gpurun_out/tf_tests.log 2>&1; tail -1 gpurun_out/tf_tests.log
AFL_NATIVE_SO=attackfl_amd/_C_pipe.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_transformer.py > gpurun_out/tf_tests2.log 2>&1; tail -1 gpurun_out/tf_tests2.log
echo "== A tree (head loss off the critical path) vs B prev"; bash tools/ab_native.sh attackfl_amd/_C_prev.so 3 --steps 20 --warmup 3 || exit 1
echo "== A tree vs B pipelined granule poll"; bash tools/ab_native.sh attackfl_amd/_C_pipe.so 3 --steps 20 --warmup 3 || exit 1
