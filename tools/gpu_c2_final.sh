#!/bin/bash
# GPU call: C2 rocprof stats + PMC passes (tools/gpu_profile.sh), then two 200-step C2
# bench lines, on the current tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c2f
export TMPDIR=/tmp
WORKLOAD=c2 bash tools/gpu_profile.sh > gpurun_out/c2f/prof.summary 2>&1 || { tail -5 gpurun_out/c2f/prof.summary; exit 1; }
tail -3 gpurun_out/c2f/prof.summary
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --workload c2 --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/c2f/b$i.json 2> gpurun_out/c2f/b$i.err || { tail -5 gpurun_out/c2f/b$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c2f/b$i.json').read().strip().splitlines()[-1])
print(round(d['ms_per_step']*1000,1), 'us/step', '%.3e' % d['value'], d.get('tick_hbm_frac'))"
done
