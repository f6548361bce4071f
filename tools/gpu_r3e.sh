#!/bin/bash
# round 3: store-update tests + C4 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py -k "c4 or store_apply or upsert or configs0 or update or insert or rejected or pinned" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_r3e.log 2>&1
s=$?; grep -E "passed|failed|error" gpurun_out/pytest_r3e.log | tail -3; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r3e.log | head -40; exit $s; }
timeout -k 10 400 python bench.py --workload c4 --steps 20 --no-cpu-baseline --no-extra > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
s=$?; python -c "
import json; d=json.loads(open('gpurun_out/bench_c4.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'])"; [ $s -ne 0 ] && { tail -20 gpurun_out/bench_c4.err; exit $s; }
exit 0
