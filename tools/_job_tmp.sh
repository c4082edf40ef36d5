set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_transformer.py tests/test_gpu_chunked.py > gpurun_out/tf_tests.log 2>&1; tail -3 gpurun_out/tf_tests.log
echo "== TF: A tree (small units on leaders, U3 2 entries) vs B prev"; bash tools/ab_native.sh attackfl_amd/_C_prev.so 3 --steps 20 --warmup 3 || exit 1
rm -f gpurun_out/ph_tf.txt
for wv in 0 4; do timeout -k 10 120 python tools/phase_profile.py --block 2 --wave $wv 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/ph_tf.txt || exit 1; done
