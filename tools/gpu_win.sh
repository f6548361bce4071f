#!/bin/bash
# GPU call: round-2 window -- large-path and parity tests, then C2's large class alone
# and the whole C2 tick, base build against the current one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/win
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_large_gpu.py tests/test_general_gpu.py tests/test_parity_gpu.py -m gpu -x -q -s --timeout 180 --timeout-method thread ${SEL:+-k "$SEL"} > gpurun_out/win/pytest.log 2>&1
s=$?; grep -E "passed|failed|round-2 window" gpurun_out/win/pytest.log | tail -4; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/win/pytest.log | head -30; exit $s; }
B=doorman_amd/libdoorman_hip_base.so
L=doorman_amd/libdoorman_hip.so
timeout -k 10 300 python -u tools/large_probe.py --steps 30 $B $L $B $L > gpurun_out/win/probe.log 2>&1 || { tail -5 gpurun_out/win/probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/win/probe.log
timeout -k 10 400 python -u tools/ab.py --workload c2 --rounds 8 --steps 20 --per-kernel $B $L > gpurun_out/win/ab.log 2>&1 || { tail -5 gpurun_out/win/ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/win/ab.log | tail -6
