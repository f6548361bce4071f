#!/bin/bash
# GPU call (round 6): the GPU test suite (optional), a size sweep (optional), then
# bench lines for the given workloads.  Every step has its own limit; the first
# failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6check}
mkdir -p $OUT
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} \
    > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 1; }
  tail -2 $OUT/gpu_tests.txt
fi
if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 400 python -u tools/size_sweep.py 20000000 $SWEEP > $OUT/size_sweep.jsonl 2> $OUT/size_sweep.err || { tail -5 $OUT/size_sweep.err; exit 1; }
  cat $OUT/size_sweep.jsonl | cut -c1-110
fi
for w in ${BENCH:-}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline $BENCHARGS \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -8 $OUT/bench_$w.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1])
print('$w', round(d['ms_per_step']*1e3, 2), 'us', {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
