#!/bin/bash
# GPU call: C2's large class alone: base, current, current without the window.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/win
export TMPDIR=/tmp
B=doorman_amd/libdoorman_hip_base.so
L=doorman_amd/libdoorman_hip.so
timeout -k 10 120 python -u -m pytest tests/test_large_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -k "window or oracle" > gpurun_out/win/pytest2.log 2>&1
s=$?; tail -1 gpurun_out/win/pytest2.log; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/win/pytest2.log | head -30; exit $s; }
timeout -k 10 300 python -u tools/large_probe.py --steps 30 $B $L $L@DM_ROUND2_WINDOW=0 $B $L $L@DM_ROUND2_WINDOW=0 ${EXTRA:-} > gpurun_out/win/probe2.log 2>&1 || { tail -5 gpurun_out/win/probe2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/win/probe2.log
