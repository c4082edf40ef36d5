#!/bin/bash
# round-4 A/B batch: HAR stem with LDS-staged parameters (tests, rocprof of the stem, bench A/B)
set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_har.py tests/test_gpu_programs.py -k "har or TransformerClassifier" > gpurun_out/t_har.log 2>&1; rc=$?; tail -2 gpurun_out/t_har.log; [ $rc -eq 0 ] || exit $rc
bash tools/rocprof_har.sh || exit 1
f=$(ls gpurun_out/prof_har/*kernel_stats.csv gpurun_out/prof_har/*/*kernel_stats.csv 2>/dev/null | head -1); python tools/rocprof_summary.py "$f" "HAR TransformerClassifier, round 4 final tree: rocprofv3 --kernel-trace --stats, bench.py --steps 1 --warmup 1" 20 > gpurun_out/prof_har_summary.md 2>&1 || true
grep -E "stem|post_bwd|attn" gpurun_out/prof_har_summary.md | head -8
echo "== HAR A/B (A = new stem, B = previous build)"; timeout -k 10 600 bash tools/ab_native.sh attackfl_amd/_C_prev.so 3 --model TransformerClassifier --data-name HAR --steps 3 --warmup 1 || exit 1
