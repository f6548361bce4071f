#!/bin/bash
# round 3: hierarchy tests + the default bench + two-rank rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_hierarchy_gpu.py tests/test_hierarchy_dist_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_r3d.log 2>&1
s=$?; grep -E "passed|failed|error" gpurun_out/pytest_r3d.log | tail -3; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r3d.log | head -40; exit $s; }
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-extra > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
s=$?; python -c "
import json; d=json.loads(open('gpurun_out/bench_c3.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], d['kernels'])"; [ $s -ne 0 ] && { tail -20 gpurun_out/bench_c3.err; exit $s; }
timeout -k 10 400 python bench.py --gpus 2 --same-device --dist-backend gloo --steps 10 --no-extra > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err
s=$?; python -c "
import json; d=json.loads(open('gpurun_out/bench_g2.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], d['config']['leases_per_gpu'], d['config']['leases_total'], d['kernels'])"; [ $s -ne 0 ] && { tail -20 gpurun_out/bench_g2.err; exit $s; }
exit 0
