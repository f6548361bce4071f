#!/bin/bash
# (the probe libraries are built from tools/attempts/r05_queue_probes.patch applied on the round-5 source)
# GPU call (round 5): the C2 tick per assignment of the created hardware queues to the
# auxiliary streams (tools/ab_libs/perm.so, DM_EXP_PERM = aux slot of the i-th queue)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5perm}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-1}); do
  for pv in ${PERMS}; do  # perm[:prio]
    v=${pv%%:*}; pr=${pv#*:}
    timeout -k 10 300 env DM_LIB=$PWD/tools/ab_libs/${PLIB:-perm}.so DM_EXP_PERM=$v DM_EXP_Q=$v DM_EXP_PRIO=$pr python -u tools/c2_after.py > $OUT/${v}${pr}_$r.txt 2>&1 || { tail -5 $OUT/${v}${pr}_$r.txt; exit 1; }
    echo "$pv $(grep -v amdgpu.ids $OUT/${v}${pr}_$r.txt | tail -1)"
  done
done
