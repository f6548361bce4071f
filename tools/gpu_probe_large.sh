#!/bin/bash
# GPU call: tools/large_probe.py over builds / modes (large class alone, small
# classes alone, whole C2).  Every GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=doorman_amd/libdoorman_hip.so; V=tools/variants
: > gpurun_out/probe.log
for sel in "" "--small" "--all"; do
  timeout -k 10 200 python -u tools/large_probe.py $sel ${PROBE_LIBS:-$L $L:chain} >> gpurun_out/probe.log 2>&1 || { tail -5 gpurun_out/probe.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/probe.log
