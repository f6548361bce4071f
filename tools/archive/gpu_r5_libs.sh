#!/bin/bash
# GPU call (round 5): bench lines per library variant (tools/ab_libs/LIB.so), WORKLOADS
# each, REPS rounds interleaved; prints the step time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5libs}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS}; do
    for w in ${WORKLOADS:-c1}; do
      f=$OUT/${w}_${lib}_$rep.json
      arg=""; [ "$lib" != prod ] && arg="--lib tools/ab_libs/$lib.so"
      timeout -k 10 300 python -u bench.py --workload $w --hier off --no-cpu-baseline --no-extra $arg > $f 2> $f.err || { tail -5 $f.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$w $lib', round(d['ms_per_step']*1000, 2))"
    done
  done
done
