#!/bin/bash
# GPU call: the chain's GPU tests on the current build, then tools/gpu_swapbench.sh
# (base build against VAR, interleaved 200-step bench lines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_large_gpu.py tests/test_parity_gpu.py} > gpurun_out/check.log 2>&1 || { tail -30 gpurun_out/check.log; exit 1; }
tail -3 gpurun_out/check.log
bash tools/gpu_swapbench.sh
