#!/bin/bash
# round-3: granule hand-offs in the on-chip TransformerModel trainer — correctness, phase profile, headline bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_transformer.py tests/test_gpu_engine.py > gpurun_out/t_r3c.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/phase_profile.py --clients 8 > gpurun_out/phase_r3c.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 >> gpurun_out/b_r3c.log 2>&1 || exit 1
done
