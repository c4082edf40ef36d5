#!/bin/bash
# round-4 A/B batch: HAR attention forward / dQ workgroup size (8 / 16 waves instead of 12: 32 resident waves per CU)
set -o pipefail
for v in _C_aq8 _C_aq16; do AFL_NATIVE_SO=attackfl_amd/$v.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_har.py > gpurun_out/t_har_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 gpurun_out/t_har_$v.log)"; [ $rc -eq 0 ] || exit $rc; done
echo "== HAR A/B (A = 12 waves, B = 8 waves)"; timeout -k 10 600 bash tools/ab_native.sh attackfl_amd/_C_aq8.so 3 --model TransformerClassifier --data-name HAR --steps 3 --warmup 1 || exit 1
echo "== HAR A/B (A = 12 waves, B = 16 waves)"; timeout -k 10 600 bash tools/ab_native.sh attackfl_amd/_C_aq16.so 3 --model TransformerClassifier --data-name HAR --steps 3 --warmup 1 || exit 1
