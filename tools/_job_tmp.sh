set -o pipefail
AFL_NATIVE_SO=attackfl_amd/_C_lm.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_transformer.py > gpurun_out/tf_tests.log 2>&1; tail -1 gpurun_out/tf_tests.log
echo "== A tree vs B leaders' masks late"; bash tools/ab_native.sh attackfl_amd/_C_lm.so 4 --steps 20 --warmup 3 || exit 1
