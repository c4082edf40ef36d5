set -e -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_transformer.py tests/test_gpu_rnn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_both.log 2>&1
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/b3_$i.log 2>&1; done
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --model RNNModel > gpurun_out/b_rnn$i.log 2>&1; done
