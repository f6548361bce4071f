#!/bin/bash
# GPU call: the C2 bench line (200 steps, one context per process) with CUs reserved
# for the large chain's stream (DM_CU_RESERVE), interleaved with the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c2res
export TMPDIR=/tmp
for v in ${VALS:-0 64 128 0 64 128}; do
  DM_CU_RESERVE=$v timeout -k 10 200 python -u bench.py --workload c2 --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/c2res/b.json 2> gpurun_out/c2res/b.err || { tail -3 gpurun_out/c2res/b.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c2res/b.json').read().strip().splitlines()[-1])
print('reserve $v', round(d['ms_per_step']*1000,1), 'us')"
done
