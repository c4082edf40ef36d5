#!/bin/bash
# rocprofv3 kernel traces of the final round-5 tree: TransformerModel headline, RNNModel, CNNModel (bench.py,
# 10 timed rounds), for per-kernel stats and round gaps (tools/rocprof_summary.py, tools/round_gaps.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for m in TransformerModel RNNModel CNNModel; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final_$m -o run -- \
    python3 $R/bench.py --model $m --steps 10 --warmup 2 > $R/gpurun_out/prof_final_$m.log 2>&1 || exit $?
done
echo prof-done
