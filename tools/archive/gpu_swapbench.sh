#!/bin/bash
# GPU call: bench.py lines (one context per process) for the base build and a variant
# swapped in turn into doorman_amd/libdoorman_hip.so on the box (WL workload, N steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/swap
export TMPDIR=/tmp
cp doorman_amd/libdoorman_hip.so /tmp/cur.so
for i in 1 2 3; do
for L in doorman_amd/libdoorman_hip_base.so $VAR; do
  cp $L doorman_amd/libdoorman_hip.so
  timeout -k 10 200 python -u bench.py --workload ${WL:-c2} --steps ${N:-200} --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/swap/b.json 2> gpurun_out/swap/b.err || { tail -5 gpurun_out/swap/b.err; cp /tmp/cur.so doorman_amd/libdoorman_hip.so; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/swap/b.json').read().strip().splitlines()[-1])
print('$(basename $L)', round(d['ms_per_step']*1000,1), 'us/step', {k: v['avg_us'] for k, v in d.get('kernels', {}).items()})"
done; done
cp /tmp/cur.so doorman_amd/libdoorman_hip.so
