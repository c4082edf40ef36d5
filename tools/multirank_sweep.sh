#!/bin/bash
# Multi-rank rounds/s on ONE GPU: world 1 vs N ranks sharing the device (gloo group, one-shot IPC
# all-gather, replicated validation, speculative launch), for the BASELINE configurations that matter at
# world > 1.  One JSON line per run in $OUT (default gpurun_out/multirank.jsonl); each run is bounded.
#   bash tools/multirank_sweep.sh [steps] [warmup]
set -o pipefail
STEPS=${1:-20}
WARM=${2:-5}
OUT=${OUT:-gpurun_out/multirank.jsonl}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
PORT=29611
run() {  # world, extra bench args...
  local w=$1; shift
  local line
  if [ "$w" = 1 ]; then
    line=$(timeout -k 10 240 python bench.py --steps "$STEPS" --warmup "$WARM" "$@" 2>/dev/null | grep '^{') || return 1
  else
    PORT=$((PORT + 1))
    line=$(AFL_BENCH_DEVICE=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$w" \
      --master-addr 127.0.0.1 --master-port $PORT bench.py --gpus "$w" --steps "$STEPS" --warmup "$WARM" "$@" \
      2>/dev/null | grep '^{') || return 1
  fi
  echo "$line" >> "$OUT"
  echo "world=$w $* -> $(echo "$line" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["comm"])')"
}
for cfg in "" "--attackers 3:LIE:2:0.74" "--mode hyper --model RNNModel --attackers 6:Opt-Fang:2"; do
  for w in 1 2 8; do
    # shellcheck disable=SC2086
    run $w $cfg || exit 1
  done
done
