#!/bin/bash
# GPU call: configs[4]'s bench line with asynchronous store batches (default) and with the
# synchronous dm_store_apply, alternated twice.  Every step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c4async
mkdir -p $OUT
for r in 1 2; do
  for mode in async sync; do
    extra=$([ $mode = sync ] && echo --c4-sync-apply || true)
    timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --no-cpu-baseline $extra > $OUT/${mode}_$r.json 2> $OUT/${mode}_$r.err || { tail -5 $OUT/${mode}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${mode}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$mode', '$r', round(d['ms_per_step'], 3), 'ms', r['kernel'], r['avg_launch_us'], r['frac'], 'busy', r['busy_gpu']['avg_launch_us'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
  done
done
