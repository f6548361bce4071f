#!/bin/bash
# GPU call: the staged-templates hop as stream memory -- hierarchy tests with the
# exchange on its own stream at G = 1 (DM_HIER_XSTREAM=1) and with the event form,
# then the C3 step for one stream / two streams + value hop / two streams + event hop.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/xs2
export TMPDIR=/tmp
for v in "DM_HIER_XSTREAM=1" "DM_HIER_XSTREAM=1 DM_XS_READY_VALUE=1" "DM_HIER_XSTREAM=0"; do
  env $v timeout -k 10 300 python -u -m pytest tests/test_hierarchy_gpu.py tests/test_hierarchy_dist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xs2/pytest.log 2>&1
  s=$?; echo "[$v] $(tail -1 gpurun_out/xs2/pytest.log)"; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/xs2/pytest.log | head -30; exit $s; }
done
for v in "DM_HIER_XSTREAM=0" "DM_HIER_XSTREAM=1" "DM_HIER_XSTREAM=1 DM_XS_READY_VALUE=1" "DM_HIER_XSTREAM=0" "DM_HIER_XSTREAM=1" "DM_HIER_XSTREAM=1 DM_XS_READY_VALUE=1"; do
  env $v timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/xs2/b.json 2> gpurun_out/xs2/b.err || { tail -5 gpurun_out/xs2/b.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/xs2/b.json').read().strip().splitlines()[-1])
print('[$v]', round(d['ms_per_step']*1000,1), 'us/step', {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
