#!/bin/bash
# A/B: CU partitions of the auxiliary streams on C2 (DM_CU_PART)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for part in none 115,26,56,59 96,40,60,60 80,48,64,64 none 128,32,48,48; do
  if [ $part = none ]; then unset DM_CU_PART; else export DM_CU_PART=$part; fi
  timeout -k 10 200 python bench.py --workload c2 --steps 50 --no-cpu-baseline --no-extra > gpurun_out/cupart_$part.json 2>/dev/null || exit $?
  python -c "
import json,sys; d=json.loads(open('gpurun_out/cupart_$part.json').read().strip().splitlines()[-1])
print('$part', round(d['ms_per_step']*1000,1), 'us/tick')"
done
