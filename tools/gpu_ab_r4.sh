#!/bin/bash
# round-4 A/B batch: HAR weight-image build with 4 k per thread (tests, rocprof, bench A/B)
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_har.py tests/test_gpu_programs.py -k "har or TransformerClassifier" > gpurun_out/t_har.log 2>&1; rc=$?; tail -1 gpurun_out/t_har.log; [ $rc -eq 0 ] || exit $rc
bash tools/rocprof_har.sh || exit 1
f=$(ls gpurun_out/prof_har/*kernel_stats.csv gpurun_out/prof_har/*/*kernel_stats.csv 2>/dev/null | head -1); python tools/rocprof_summary.py "$f" "HAR" 30 > gpurun_out/prof_har_summary.md 2>&1 || true
grep -E "post|qkv" gpurun_out/prof_har_summary.md | head -4
echo "== HAR A/B (A = new, B = previous build)"; timeout -k 10 600 bash tools/ab_native.sh attackfl_amd/_C_prev.so 3 --model TransformerClassifier --data-name HAR --steps 3 --warmup 1 || exit 1
