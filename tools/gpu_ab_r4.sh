#!/bin/bash
# round-4 A/B batch: HAR q|k|v forward at 16 waves per workgroup (A) vs 8 (B = previous build)
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_har.py tests/test_gpu_programs.py -k "har or TransformerClassifier" > gpurun_out/t_har.log 2>&1; rc=$?; tail -1 gpurun_out/t_har.log; [ $rc -eq 0 ] || exit $rc
bash tools/rocprof_har.sh || exit 1
f=$(ls gpurun_out/prof_har/*kernel_stats.csv gpurun_out/prof_har/*/*kernel_stats.csv 2>/dev/null | head -1); python tools/rocprof_summary.py "$f" "HAR" 30 > gpurun_out/prof_har_summary.md 2>&1 || true
grep -E "k_har_qkv" gpurun_out/prof_har_summary.md | head -4
args="--model TransformerClassifier --data-name HAR --steps 3 --warmup 1"
for i in 1 2 3; do
  a=$(timeout -k 10 150 python bench.py $args 2>/dev/null | grep '^{' | python -c 'import json,sys; print(json.load(sys.stdin)["value"])') || exit 1
  b=$(AFL_NATIVE_SO=attackfl_amd/_C_prev.so timeout -k 10 150 python bench.py $args 2>/dev/null | grep '^{' | python -c 'import json,sys; print(json.load(sys.stdin)["value"])') || exit 1
  echo "A $a  B $b"
done
