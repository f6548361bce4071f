#!/bin/bash
# GPU call: hierarchy tests, then the C3 step (hier_root event time) with the base build
# and the current one swapped in turn into doorman_amd/libdoorman_hip.so (box copy only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/hier
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hierarchy_gpu.py tests/test_hierarchy_dist_gpu.py tests/test_server_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/hier/pytest.log 2>&1
s=$?; tail -1 gpurun_out/hier/pytest.log; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/hier/pytest.log | head -30; exit $s; }
cp doorman_amd/libdoorman_hip.so /tmp/cur.so
for i in 1 2; do
for L in doorman_amd/libdoorman_hip_base.so /tmp/cur.so; do
  cp $L doorman_amd/libdoorman_hip.so
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/hier/b.json 2> gpurun_out/hier/b.err || { tail -5 gpurun_out/hier/b.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/hier/b.json').read().strip().splitlines()[-1])
print('$L', round(d['ms_per_step']*1000,1), 'us/step', {k: v['avg_us'] for k, v in d['kernels'].items()})"
done; done
cp /tmp/cur.so doorman_amd/libdoorman_hip.so
