#!/bin/bash
# round 3: the dense split of the 256x8 / 512x8 bins -- tests + interleaved A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py -k "dense or random_all_bins or c1 or c2 or c3" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_r3f.log 2>&1
s=$?; [ "${SKIP_TESTS:-0}" = 1 ] || grep -E "passed|failed|error" gpurun_out/pytest_r3f.log | tail -3; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r3f.log | head -40; exit $s; }
L=doorman_amd/libdoorman_hip.so
for w in ${AB_WORKLOADS:-c3 c2 c1}; do
  timeout -k 10 300 python tools/ab.py --workload $w --rounds 6 --steps 20 --per-kernel "$L@DM_DENSE_SPLIT=3" "$L@DM_DENSE_SPLIT=1" "$L@DM_DENSE_SPLIT=0" > gpurun_out/ab_dense_$w.txt 2>&1 || { tail -20 gpurun_out/ab_dense_$w.txt; exit 1; }
  cat gpurun_out/ab_dense_$w.txt
done
exit 0
