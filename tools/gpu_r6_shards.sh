#!/bin/bash
# GPU call (round 6, final tree): one rank's step of an N = 2 / 4 / 8 configs[3] node
# (bench.py --rehearse-shard N), twice each.  Every step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r6shards
mkdir -p $OUT
for r in 1 2; do
  for n in 8 4 2; do
    timeout -k 10 300 python -u bench.py --rehearse-shard $n --steps 200 --warmup 20 --no-cpu-baseline > $OUT/shard${n}_$r.json 2> $OUT/shard${n}_$r.err || { tail -5 $OUT/shard${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/shard${n}_$r.json').read().strip().splitlines()[-1]); print($n, '$r', round(d['ms_per_step']*1e3, 2), d.get('dist', {}).get('consistent'))"
  done
done
