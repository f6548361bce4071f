#!/bin/bash
# GPU call: the whole GPU suite, smoke(), the C2 and default bench lines and the C2
# rocprofv3 evidence (tools/gpu_profile.sh) on the current tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4final
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -20 $OUT/gpu_tests.txt; exit 1; }
tail -2 $OUT/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 300 python -u bench.py --workload c2 --steps 50 --warmup 10 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -5 $OUT/bench_c2.err; exit 1; }
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "
import json
for n in ('c2', 'default'):
    d = json.loads(open('$OUT/bench_%s.json' % n).read().strip().splitlines()[-1])
    print(n, d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
if [ "${PROFILE:-1}" = 1 ]; then WORKLOAD=c2 bash tools/gpu_profile.sh; fi
