set -e -o pipefail
true
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --model RNNModel > gpurun_out/b_rnn$i.log 2>&1; done
