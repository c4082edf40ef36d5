#!/bin/bash
# world-2 headline repeats (two ranks sharing one GPU), with per-round host timings of rank 0
set -o pipefail
for i in 1 2 3; do
  line=$(AFL_BENCH_DEVICE=0 AFL_BENCH_TIMES=gpurun_out/mr2_times_$i.jsonl timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29800 + i)) bench.py --gpus 2 --steps 20 --warmup 5 2>gpurun_out/mr2_$i.err | grep '^{') || { tail -20 gpurun_out/mr2_$i.err; exit 1; }
  echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print("world=2", d["value"], d["comm"], d["config"]["trainer"], d["speculative"])'
done
line=$(timeout -k 10 240 python bench.py --steps 20 --warmup 5 2>/dev/null | grep '^{') || exit 1
echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print("world=1", d["value"], d["comm"], d["config"]["trainer"], d["speculative"])'
