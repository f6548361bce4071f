#!/bin/bash
# C2: enqueue order A/B (DM_LARGE_LAST)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 1 0 1; do
  DM_LARGE_LAST=$v timeout -k 10 200 python bench.py --workload c2 --steps 100 --no-cpu-baseline --no-extra > gpurun_out/c2o_$v.json 2>/dev/null || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/c2o_$v.json').read().strip().splitlines()[-1])
print('large_last $v', round(d['ms_per_step']*1000,1), 'us/tick')"
done
