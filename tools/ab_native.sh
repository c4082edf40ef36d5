#!/bin/bash
# A/B two native builds on the same box: alternates bench.py runs of attackfl_amd/_C.so (A) and the
# variant $1 (B, loaded through AFL_NATIVE_SO), N times each.  Extra args go to bench.py.
#   bash tools/ab_native.sh attackfl_amd/_C_ab.so 3 --steps 30 --warmup 5
set -o pipefail
VAR=$1; N=${2:-3}; shift 2
for i in $(seq 1 "$N"); do
  a=$(timeout -k 10 120 python bench.py "$@" 2>/dev/null | grep '^{' | python -c 'import json,sys; print(json.load(sys.stdin)["value"])') || exit 1
  b=$(AFL_NATIVE_SO=$VAR timeout -k 10 120 python bench.py "$@" 2>/dev/null | grep '^{' | python -c 'import json,sys; print(json.load(sys.stdin)["value"])') || exit 1
  echo "A $a  B $b"
done
