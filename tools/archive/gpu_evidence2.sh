#!/bin/bash
# GPU call: rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes per workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${PROF_WORKLOADS:-c3 c2 c1}; do
  WORKLOAD=$w bash tools/gpu_profile.sh > gpurun_out/prof_$w.summary 2>&1 || { tail -5 gpurun_out/prof_$w.summary; exit 1; }
  tail -3 gpurun_out/prof_$w.summary
done
