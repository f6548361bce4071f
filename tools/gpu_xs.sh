#!/bin/bash
# GPU call: cross-stream signals (stream memory ops) -- hierarchy / dist / parity tests,
# the stream-memory (DM_XS_VALUES) form's hierarchy tests, the pipelined-step probe and the C3 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/xs
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hierarchy_gpu.py tests/test_hierarchy_dist_gpu.py tests/test_parity_gpu.py tests/test_large_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xs/pytest.log 2>&1
s=$?; tail -2 gpurun_out/xs/pytest.log; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/xs/pytest.log | head -30; exit $s; }
DM_XS_VALUES=1 timeout -k 10 300 python -u -m pytest tests/test_hierarchy_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xs/pytest_ev.log 2>&1
s=$?; tail -1 gpurun_out/xs/pytest_ev.log; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/xs/pytest_ev.log | head -30; exit $s; }
timeout -k 10 200 python -u tools/pipe_probe.py > gpurun_out/xs/pipe.log 2>&1 || { tail -5 gpurun_out/xs/pipe.log; exit 1; }
grep "us/step" gpurun_out/xs/pipe.log
for v in "" "--no-pipeline" "--hier off"; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-extra $v > gpurun_out/xs/b.json 2> gpurun_out/xs/b.err || { tail -5 gpurun_out/xs/b.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/xs/b.json').read().strip().splitlines()[-1])
print('[$v]', round(d['ms_per_step']*1000,1), 'us/step', {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
