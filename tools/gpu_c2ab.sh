#!/bin/bash
# GPU call: interleaved C2 tick A/B of the base build against variants (VARS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c2ab
export TMPDIR=/tmp
B=doorman_amd/libdoorman_hip_base.so
timeout -k 10 500 python -u tools/ab.py --workload c2 --rounds ${ROUNDS:-8} --steps 20 ${PK:-} $B $VARS > gpurun_out/c2ab/ab.log 2>&1 || { tail -5 gpurun_out/c2ab/ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c2ab/ab.log | tail -12
