#!/bin/bash
# C2: two-chain split A/B + its tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DM_LARGE_STREAMS=2 timeout -k 10 400 python -u -m pytest tests/test_large_gpu.py tests/test_general_gpu.py "tests/test_parity_gpu.py::test_c2_zipf_full_size_sampled" "tests/test_parity_gpu.py::test_random_all_bins" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_c2ab.log 2>&1
s=$?; tail -2 gpurun_out/pytest_c2ab.log; [ $s -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/pytest_c2ab.log | head -20; exit $s; }
for v in 1 2 1 2; do
  DM_LARGE_STREAMS=$v timeout -k 10 200 python bench.py --workload c2 --steps 100 --no-cpu-baseline --no-extra > gpurun_out/c2ab_$v.json 2>/dev/null || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/c2ab_$v.json').read().strip().splitlines()[-1])
print('streams $v', round(d['ms_per_step']*1000,1), 'us/tick')"
done
