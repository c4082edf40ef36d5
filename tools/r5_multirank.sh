#!/bin/bash
# Round-5 regression check of the multi-rank path on one GPU (N ranks sharing the device): the round-4 sweep
# (tools/multirank_sweep.sh) plus CNNModel at world 1 / 2 (the round-5 CNN round boundary and sharer counting).
set -o pipefail
OUT=gpurun_out/multirank_r5.jsonl bash tools/multirank_sweep.sh 20 5 || exit 1
PORT=29711
line=$(timeout -k 10 240 python bench.py --steps 20 --warmup 5 --model CNNModel 2>/dev/null | grep '^{') || exit 1
echo "$line" >> gpurun_out/multirank_r5.jsonl; echo "world=1 CNNModel -> $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["comm"], d["config"]["trainer"])')"
line=$(AFL_BENCH_DEVICE=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port $PORT bench.py --gpus 2 --steps 20 --warmup 5 --model CNNModel 2>gpurun_out/mr_cnn2.err | grep '^{') || { tail -20 gpurun_out/mr_cnn2.err; exit 1; }
echo "$line" >> gpurun_out/multirank_r5.jsonl; echo "world=2 CNNModel -> $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["comm"], d["config"]["trainer"])')"
