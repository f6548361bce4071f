#!/bin/bash
# GPU call: the large-resource tests, then an interleaved A/B of the one-launch
# path against the chain on C2.  Every GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_large_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_large.log 2>&1
s=$?; grep -E "passed|failed|error|max \||plan" gpurun_out/pytest_large.log | tail -20; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_large.log | head -30; exit $s; }
L=doorman_amd/libdoorman_hip.so
timeout -k 10 300 python -u tools/ab.py --workload c2 --rounds ${ROUNDS:-6} --steps 20 $L $L:chain > gpurun_out/ab_large.log 2>&1
s=$?; cat gpurun_out/ab_large.log | tail -5; exit $s
