#!/bin/bash
# GPU call (round 5): the stream-parts tests, then the N=8 rehearsal step and C1 / C3
# lines with the current tree.  Every step has its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5parts}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_parts_gpu.py tests/test_hierarchy_gpu.py} -x -v --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
for w in ${BENCHES:-shard8 c1}; do
  case $w in
    shard8) args="--workload c3 --rehearse-shard 8 --steps 200 --warmup 20";;
    *) args="--workload $w --no-cpu-baseline --no-extra";;
  esac
  timeout -k 10 300 python -u bench.py $args > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -5 $OUT/bench_$w.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1])
r=d.get('rehearsal') or {}
print('$w', d['value'], d['ms_per_step'], r.get('step_us'), {k: v['avg_us'] for k, v in (d.get('kernels') or {}).items()} or (d.get('roofline') or {}).get('kernel'))"
done
