#!/bin/bash
# GPU call: where the C3 step's time goes beyond the dense kernel.  Bench lines for
# the pipelined exchange (default), the unpipelined one and no exchange; a kernel
# trace of the default step through tools/timeline.py; then C2's large class alone,
# chain against the persistent flow path (tools/large_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c3s
export TMPDIR=/tmp
for v in "" "--no-pipeline" "--hier off"; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-extra $v > gpurun_out/c3s/b.json 2> gpurun_out/c3s/b.err || { tail -5 gpurun_out/c3s/b.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c3s/b.json').read().strip().splitlines()[-1])
print('[$v]', round(d['ms_per_step']*1000,1), 'us/step', {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/c3s/trace -o run -- python3 bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/c3s/tl_log.txt 2>&1 || { tail -5 gpurun_out/c3s/tl_log.txt; exit 1; }
python3 tools/timeline.py gpurun_out/c3s/trace --skip 20 > gpurun_out/c3s/timeline.txt 2>&1; tail -30 gpurun_out/c3s/timeline.txt
L=doorman_amd/libdoorman_hip.so
timeout -k 10 300 python -u tools/large_probe.py --steps 30 $L@DM_LARGE_PATH=0 $L@DM_LARGE_PATH=2,DM_FLOW_WG=2 $L@DM_LARGE_PATH=2,DM_FLOW_WG=4 $L@DM_LARGE_PATH=0 > gpurun_out/c3s/flow.log 2>&1
s=$?; grep -v amdgpu.ids gpurun_out/c3s/flow.log | tail -20; exit $s
