#!/bin/bash
# GPU call (round 5, probe): the N=8 rehearsal step with CUs reserved for the exchange
# (tools/ab_libs/res.so: DM_PROBE_RESERVE CUs left out of the library's streams; the
# exchange stream masked to them, DM_PROBE_HIER=xres)
# (round-5 probe: the probe builds come from tools/attempts/r05_parts_exchange_probes.patch /
#  r05_queue_probes.patch applied on the round-5 source; results in profiles/r05_parts_ab.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5res
for rep in 1 2; do
for k in ${KS:-0 8 16 32}; do
  if [ $k = 0 ]; then pre="DM_PROBE_HIER=none"; else pre="DM_PROBE_HIER=xres DM_PROBE_RESERVE=$k"; fi
  f=gpurun_out/r5res/res${k}_$rep.json
  env $pre timeout -k 10 200 python -u bench.py --workload c3 --rehearse-shard 8 --steps 200 --warmup 20 --lib tools/ab_libs/res.so > $f 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('reserve $k', d['rehearsal']['step_us'], d.get('host_enqueue_us_per_step'), {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
done
