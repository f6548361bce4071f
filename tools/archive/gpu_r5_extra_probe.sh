#!/bin/bash
# GPU call (round 5): why the default run's configs[2] extra line is slower than a C2
# run of its own -- the default run with and without the CPU baseline before the extras.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5probe
mkdir -p $OUT
for v in "nocpu:--no-cpu-baseline" "cpu:"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 600 python -u bench.py $a > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { tail -5 $OUT/bench_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/bench_$n.json').read().strip().splitlines()[-1])
for k,v in d['extra'].items(): print('$n', k, v['ms_per_step'], v.get('host_enqueue_us_per_step'))"
done
