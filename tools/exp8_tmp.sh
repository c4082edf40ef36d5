#!/bin/bash
set -o pipefail
P=29700
r() { P=$((P+1)); echo "== $*"; env AFL_BENCH_DEVICE=0 "$@" timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 8 --steps 20 --warmup 5 2>/dev/null | grep '^{' | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["comm"], d["ms_per_step"])'; }
r GPU_MAX_HW_QUEUES=1
r GPU_MAX_HW_QUEUES=2
r GPU_MAX_HW_QUEUES=4 AFL_BENCH_ONE_SHOT=false
r GPU_MAX_HW_QUEUES=1 AFL_BENCH_ONE_SHOT=false
