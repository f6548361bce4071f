#!/bin/bash
# GPU call: the persistent large path's tests, then an interleaved A/B on C2 of the
# chain against the persistent path (grid variants).  Every GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_large_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread ${SEL:+-k "$SEL"} > gpurun_out/pytest_flow.log 2>&1
s=$?; grep -E "passed|failed|error|max \|" gpurun_out/pytest_flow.log | tail -30; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_flow.log | head -30; exit $s; }
L=doorman_amd/libdoorman_hip.so
timeout -k 10 400 python -u tools/ab.py --workload ${WL:-c2} --rounds ${ROUNDS:-6} --steps 20 --per-kernel ${VARIANTS:-$L@DM_LARGE_PATH=0 $L@DM_LARGE_PATH=2,DM_FLOW_WG=2 $L@DM_LARGE_PATH=2,DM_FLOW_WG=4} > gpurun_out/ab_flow.log 2>&1
s=$?; tail -40 gpurun_out/ab_flow.log; exit $s
