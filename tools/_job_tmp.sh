set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_programs.py tests/test_gpu_chunked.py -k "cnn or CNN" > gpurun_out/cnn_tests.log 2>&1; tail -1 gpurun_out/cnn_tests.log
echo "== CNN: A tree (head loss) vs B prev"; bash tools/ab_native.sh attackfl_amd/_C_prev.so 3 --steps 20 --warmup 3 --model CNNModel || exit 1
for v in p1 p2; do
AFL_NATIVE_SO=attackfl_amd/_C_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_transformer.py > gpurun_out/tf_tests_$v.log 2>&1; tail -1 gpurun_out/tf_tests_$v.log
echo "== TF: A tree vs B pipelined poll $v"; bash tools/ab_native.sh attackfl_amd/_C_$v.so 3 --steps 20 --warmup 3 || exit 1
done
