#!/bin/bash
# GPU call (round 5): the whole GPU suite, smoke(), and the default bench line (with its
# extra c1 / c2 / c4 lines) on the current tree.  Every step has its own time limit and
# the call stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5suite}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 1; }
tail -2 $OUT/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])
for k, v in (d.get('extra') or {}).items():
    r = v.get('roofline') or {}
    print(k, v.get('value'), v.get('ms_per_step'), v.get('tick_hbm_frac'), r.get('kernel'), r.get('frac'), r.get('traffic'), r.get('algorithmic_bytes_per_launch'))"
fi
