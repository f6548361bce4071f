#!/bin/bash
# One GPU call's worth of round evidence: parity tests, smoke, every bench
# workload, and the rocprofv3 kernel-trace + PMC passes for c1 (and c3, c2).
# Every GPU step has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
s=$?; tail -3 gpurun_out/pytest_gpu.log; [ $s -ne 0 ] && exit $s
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
s=$?; tail -2 gpurun_out/smoke.log; [ $s -ne 0 ] && exit $s
bash tools/bench_all.sh || exit $?
for w in ${PROF_WORKLOADS:-c1 c3 c2}; do
  WORKLOAD=$w bash tools/gpu_profile.sh > gpurun_out/prof_$w.summary 2>&1 || { tail -5 gpurun_out/prof_$w.summary; exit 1; }
  tail -3 gpurun_out/prof_$w.summary
done
