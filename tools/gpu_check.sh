#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-30}
WORKLOAD=${WORKLOAD:-c1}
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -x -q --timeout 120 --timeout-method thread"}

stop_if_fatal() {  # $1 = exit status, $2 = step
  case "$1" in
    0|1) return 0 ;;  # ok / test failures: keep going
    *) echo "STOP after $2 (status $1)"; exit "$1" ;;
  esac
}

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
  s=$?; tail -5 gpurun_out/pytest_gpu.log; stop_if_fatal $s pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  s=$?; tail -3 gpurun_out/smoke.log; stop_if_fatal $s smoke
fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 --workload $WORKLOAD > gpurun_out/bench_$WORKLOAD.json 2> gpurun_out/bench_$WORKLOAD.err
s=$?; cat gpurun_out/bench_$WORKLOAD.json; tail -3 gpurun_out/bench_$WORKLOAD.err; stop_if_fatal $s bench
if [ "${SKIP_PROF:-0}" != 1 ]; then
  rm -rf gpurun_out/prof_$WORKLOAD
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$WORKLOAD -o run -- \
    python3 bench.py --steps $STEPS --warmup 5 --workload $WORKLOAD --no-cpu-baseline > gpurun_out/prof_$WORKLOAD.log 2>&1
  s=$?; tail -3 gpurun_out/prof_$WORKLOAD.log; stop_if_fatal $s rocprof
  find gpurun_out/prof_$WORKLOAD -name "*kernel_stats.csv" -exec cat {} \; | head -20
fi
