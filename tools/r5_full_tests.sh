#!/bin/bash
# The whole GPU suite (one process), then smoke() and the default bench.
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite_r5.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_suite_r5.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r5.log 2>&1 || exit $?
tail -2 gpurun_out/smoke_r5.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default_r5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default_r5.log
exit $rc
