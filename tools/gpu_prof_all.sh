#!/bin/bash
# round-3 evidence: rocprof stats + PMC passes for c3, c1, c2 (tools/gpu_profile.sh each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for w in c3 c1 c2; do
  WORKLOAD=$w STEPS=30 bash tools/gpu_profile.sh > gpurun_out/prof_$w.summary 2>&1 || { echo "profile $w failed"; tail -5 gpurun_out/prof_$w.summary; exit 1; }
  echo "profile $w ok"
done
mkdir -p gpurun_out/profiles_new && cp profiles/pmc_c*.json profiles/rocprof_c*.md gpurun_out/profiles_new/
