#!/bin/bash
# GPU call (round 5): one rank's step of an N-GPU configs[3] node rehearsed on one GPU
# (bench.py --rehearse-shard N), alternating library builds (LIBS, tools/ab_libs names;
# "prod" = the in-tree build) for REPS rounds; prints each run's step time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5shard}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-3}); do
  for lib in ${LIBS:-prod}; do
    arg=""; [ "$lib" != prod ] && arg="--lib tools/ab_libs/$lib.so"
    f=$OUT/shard${N:-8}_${lib}_$rep.json
    timeout -k 10 300 python -u bench.py --workload c3 --rehearse-shard ${N:-8} --steps ${STEPS:-200} --warmup 20 $arg > $f 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$lib', $rep, d['rehearsal']['step_us'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
  done
done
