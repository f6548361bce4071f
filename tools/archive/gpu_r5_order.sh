#!/bin/bash
# (the probe libraries are built from tools/attempts/r05_queue_probes.patch applied on the round-5 source)
# GPU call (round 5): the C2 tick per library variant (stream creation order / queue count
# probes), each in a fresh process, ROUNDS rounds interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5order}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-base o1}; do
    timeout -k 10 300 env DM_LIB=$PWD/tools/ab_libs/$v.so python -u tools/c2_after.py ${PRE:-} > $OUT/${v}_$r.txt 2>&1 || { tail -5 $OUT/${v}_$r.txt; exit 1; }
    grep -v amdgpu.ids $OUT/${v}_$r.txt | tail -1
  done
done
