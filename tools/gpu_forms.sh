#!/bin/bash
# GPU call: the whole GPU suite under the non-default forms (cross-stream tokens as
# stream memory + the exchange on its own stream at G = 1; the one-kernel form of the
# workgroup bins; separate sub-wave launches and plain auxiliary streams).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/forms
export TMPDIR=/tmp
for v in "DM_XS_VALUES=1 DM_HIER_XSTREAM=1" "DM_DENSE_SPLIT=0" "DM_MERGE_SUBS=0 DM_CUMASK=0"; do
  env $v timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/forms/pytest.log 2>&1
  s=$?; echo "[$v] $(tail -1 gpurun_out/forms/pytest.log)"; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/forms/pytest.log | head -30; exit $s; }
done
