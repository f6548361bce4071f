#!/bin/bash
# GPU call (round 5): the N=8 rehearsal step per stream choice of the hierarchy
# (DM_PROBE_HIER, a probe build of doorman_amd/hierarchy.py), REPS rounds interleaved
# (round-5 probe: the probe builds come from tools/attempts/r05_parts_exchange_probes.patch /
#  r05_queue_probes.patch applied on the round-5 source; results in profiles/r05_parts_ab.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5hprobe}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARS:-base}; do
    f=$OUT/${v}_$rep.json
    timeout -k 10 300 env DM_PROBE_HIER=$v python -u bench.py --workload c3 --rehearse-shard ${N:-8} --steps ${STEPS:-200} --warmup 20 > $f 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$v', $rep, d['rehearsal']['step_us'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
  done
done
