set -o pipefail
AFL_NATIVE_SO=attackfl_amd/_C_unr.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_transformer.py > gpurun_out/tf_tests.log 2>&1; tail -1 gpurun_out/tf_tests.log
echo "== A tree vs B dW loops unrolled"; bash tools/ab_native.sh attackfl_amd/_C_unr.so 3 --steps 20 --warmup 3 || exit 1
