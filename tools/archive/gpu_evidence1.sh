#!/bin/bash
# GPU call: every GPU test, smoke, every bench workload (tools/bench_all.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
s=$?; tail -3 gpurun_out/pytest_gpu.log; [ $s -ne 0 ] && exit $s
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
s=$?; tail -2 gpurun_out/smoke.log; [ $s -ne 0 ] && exit $s
bash tools/bench_all.sh
