#!/bin/bash
# GPU call (round 5, probe): the N=8 rehearsal step with two, three and four ticks of template
# lag (DM_PROBE_LAG in a probe build of doorman_amd/hierarchy.py, template slots from a
# DM_TPL_SLOTS=6 library build)
# (round-5 probe: the probe builds come from tools/attempts/r05_parts_exchange_probes.patch /
#  r05_queue_probes.patch applied on the round-5 source; results in profiles/r05_parts_ab.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5lag
for rep in 1 2; do
for cfg in "2 base" "3 slots6" "4 slots6"; do
  set -- $cfg
  DM_PROBE_LAG=$1 timeout -k 10 200 python -u bench.py --workload c3 --rehearse-shard 8 --steps 200 --warmup 20 --lib tools/ab_libs/$2.so > gpurun_out/r5lag/lag$1_$rep.json 2> gpurun_out/r5lag/lag$1_$rep.err || { tail -5 gpurun_out/r5lag/lag$1_$rep.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r5lag/lag$1_$rep.json').read().strip().splitlines()[-1])
print('lag $1', d['rehearsal']['step_us'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
done
