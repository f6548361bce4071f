#!/bin/bash
# GPU call (round 6, final tree): the GPU test suite, smoke(), then the default bench
# line (C3 north star + the C1/C2/C4 extras with the CPU baseline).  Every step has its
# own limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6final2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 1; }
tail -2 $OUT/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -8 $OUT/bench_default.err; exit 1; }
tail -c 400 $OUT/bench_default.json
