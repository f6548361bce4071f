#!/bin/bash
# GPU call: the given pytest selection (default: every GPU test), then smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SEL=${SEL:-tests}
timeout -k 10 ${TLIM:-900} python -u -m pytest $SEL -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
s=$?; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_gpu.log | head -40; exit $s; }
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  s=$?; tail -2 gpurun_out/smoke.log; exit $s
fi
