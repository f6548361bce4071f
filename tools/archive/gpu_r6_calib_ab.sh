#!/bin/bash
# GPU call: C2 bench lines with the head library and the later, interleaved queue
# calibration, alternated (each line a fresh process: its calibration from scratch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/calib_ab; mkdir -p $OUT
for r in 1 2 3; do
  for v in head calib2; do
    timeout -k 10 300 python -u bench.py --workload c2 --steps 200 --warmup 20 --no-cpu-baseline --lib tools/ab_libs/$v.so > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail -5 $OUT/${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', '$r', round(d['ms_per_step']*1e3, 2))"
  done
done
