#!/bin/bash
# Run GPU steps in order, each under its own time limit; continue past ordinary failures (test assertions), stop
# at the first fault / abort / time limit (exit 124, 134, 137, 139) so nothing more touches the GPU after it.
#   tools/gpu_seq.sh "name:secs:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "== $name"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  tail -6 "gpurun_out/$name.log" | cut -c1-300
  echo "== $name rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc ;; esac
done
