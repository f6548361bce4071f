#!/bin/bash
# GPU call: C2's large class alone, base build against variants (VARS), then (AB=1)
# the whole C2 tick.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
B=doorman_amd/libdoorman_hip_base.so
timeout -k 10 300 python -u tools/large_probe.py --steps 30 $B $VARS $B $VARS > gpurun_out/var/probe.log 2>&1 || { tail -5 gpurun_out/var/probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/var/probe.log
if [ "${AB:-0}" = 1 ]; then
timeout -k 10 400 python -u tools/ab.py --workload c2 --rounds 8 --steps 20 $B $VARS > gpurun_out/var/ab.log 2>&1 || { tail -5 gpurun_out/var/ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/var/ab.log | tail -6
fi
