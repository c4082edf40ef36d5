#!/bin/bash
# Named GPU-box recipes (run on the box through gpurun, one recipe or several in order):
#   bash tools/gpu_job.sh suite                       the whole GPU test suite (one process), smoke(), default bench
#   bash tools/gpu_job.sh tests <pytest -k expr> [files...]   a subset of the GPU tests
#   bash tools/gpu_job.sh bench [bench.py args...]     one bench line
#   bash tools/gpu_job.sh ab <variant.so> <reps> [bench args...]   A/B of attackfl_amd/_C.so against a variant build
#   bash tools/gpu_job.sh phases <tag>                 per-phase stamps, TF / RNN head + vitals branch waves 0 / 4
#   bash tools/gpu_job.sh rocprof <tag> [models...]    rocprofv3 --kernel-trace --stats of bench.py per model
#   bash tools/gpu_job.sh pmc                          the headline's PMC passes (tools/pmc_bench.sh)
#   bash tools/gpu_job.sh sweep <tag>                  every BASELINE configuration (tools/bench_configs.sh) + cliffs
#   bash tools/gpu_job.sh multirank <tag>              N ranks sharing the one GPU (tools/multirank_sweep.sh)
# Several recipes: separate them with `--`, e.g. `bash tools/gpu_job.sh suite -- phases r6 -- rocprof r6`.
# Every GPU step runs under its own time limit; the first failing step ends the job (nothing more touches the
# GPU after a fault, an abort or a time limit).  Outputs land under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out

step() {  # step <secs> <log> <command...>: bounded, output to gpurun_out/<log>, short tail to stdout
  local secs=$1 log=gpurun_out/$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  tail -3 "$log" | cut -c1-240
  return $rc
}

suite() {
  step 1100 gpu_suite.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  local rc=$?
  case $rc in 0|1) ;; *) return $rc ;; esac
  step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()" || return $?
  step 300 bench_default.log python bench.py || return $?
  return $rc
}

tests() {
  local k=$1
  shift
  step 900 tests_sel.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "$k" "${@:-tests}"
}

bench() { step 300 bench_last.log python bench.py "$@"; }

ab() {
  local so=$1 reps=$2
  shift 2
  bash tools/ab_native.sh "$so" "$reps" "$@"
}

phases() {
  local tag=${1:-last} out
  for wv in 0 4; do
    for m in TransformerModel RNNModel; do
      out=gpurun_out/phases_${m}_$tag.txt
      timeout -k 10 120 python tools/phase_profile.py --model $m --block 1 --wave $wv 2>/dev/null | grep -v amdgpu.ids >> "$out" || return 1
    done
  done
  for m in TransformerModel RNNModel; do
    timeout -k 10 120 python tools/phase_profile.py --model $m --block 0 --wave 0 2>/dev/null | grep -v amdgpu.ids \
      >> gpurun_out/phases_${m}_$tag.txt || return 1
  done
  echo phases-done
}

rocprof() {
  local tag=${1:-last}
  shift
  local models=("${@:-TransformerModel}")
  (cd /tmp && export TMPDIR=/tmp &&
    for m in "${models[@]}"; do
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${m}_$tag" -o run -- \
        python3 "$R/bench.py" --model "$m" --steps 10 --warmup 2 > "$R/gpurun_out/prof_${m}_$tag.log" 2>&1 || exit $?
    done) || return $?
  echo prof-done
}

pmc() { bash tools/pmc_bench.sh; }

sweep() {
  local tag=${1:-last}
  STEPS=30 OUT=gpurun_out/bench_configs_$tag.jsonl bash tools/bench_configs.sh || return 1
  local out=gpurun_out/cliff_$tag.jsonl args
  : > "$out"
  for args in "--model CNNModel --clients 16" "--model TransformerModel --clients 128" "--model RNNModel --clients 128"; do
    # shellcheck disable=SC2086
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 $args > gpurun_out/cliff_last.log 2>&1 || return 1
    tail -1 gpurun_out/cliff_last.log >> "$out"
  done
}

multirank() { OUT=gpurun_out/multirank_${1:-last}.jsonl bash tools/multirank_sweep.sh 20 5; }

# split "$@" on `--` into recipes and run them in order
cmd=()
run_cmd() {
  [ ${#cmd[@]} -eq 0 ] && return 0
  echo "== ${cmd[*]}"
  "${cmd[@]}"
  local rc=$?
  [ $rc -ne 0 ] && echo "== ${cmd[0]} failed (rc=$rc)"
  return $rc
}
for a in "$@"; do
  if [ "$a" = "--" ]; then
    run_cmd || exit $?
    cmd=()
  else
    cmd+=("$a")
  fi
done
run_cmd || exit $?
