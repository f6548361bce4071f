#!/bin/bash
# GPU call (round 5, probe): single-context workloads with the CU bits DM_PROBE_RESBITS
# left out of the library's auxiliary streams (tools/ab_libs/res.so), then the N=8
# rehearsal with the exchange stream masked to those CUs (DM_PROBE_HIER=xres)
# (round-5 probe: the probe builds come from tools/attempts/r05_parts_exchange_probes.patch /
#  r05_queue_probes.patch applied on the round-5 source; results in profiles/r05_parts_ab.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5res2
declare -A SETS=([none]="" [top]="248,249,250,251,252,253,254,255" [low]="0,1,2,3,4,5,6,7" [stride]="31,63,95,127,159,191,223,255" [stride8]="7,15,23,31,39,47,55,63")
for name in ${NAMES:-none top low stride stride8}; do
  bits=${SETS[$name]}
  for w in c1 c2; do
    f=gpurun_out/r5res2/${w}_$name.json
    DM_PROBE_RESBITS=$bits timeout -k 10 300 python -u bench.py --workload $w --hier off --no-cpu-baseline --no-extra --lib tools/ab_libs/res.so > $f 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$w $name', round(d['ms_per_step']*1000, 2))"
  done
  if [ -n "$bits" ]; then
    f=gpurun_out/r5res2/sh8_$name.json
    DM_PROBE_RESBITS=$bits DM_PROBE_HIER=xres timeout -k 10 200 python -u bench.py --workload c3 --rehearse-shard 8 --steps 200 --warmup 20 --lib tools/ab_libs/res.so > $f 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('shard8 $name', d['rehearsal']['step_us'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
  fi
done
