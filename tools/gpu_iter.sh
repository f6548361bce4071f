#!/bin/bash
# GPU call for one build iteration: every GPU test, then the large-path probe
# (large class alone, small classes alone, whole C2).  Each step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest ${SEL:-tests} -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  s=$?; grep -E "passed|failed|error|max \|" gpurun_out/pytest_gpu.log | tail -16; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_gpu.log | head -30; exit $s; }
fi
[ "${SKIP_PROBE:-0}" = 1 ] && exit 0
bash tools/gpu_probe_large.sh
