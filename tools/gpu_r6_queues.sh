#!/bin/bash
# GPU call (round 6): configs[2]'s tick after the process created K hardware queues of
# its own first (K = 0..3 CU-masked HIP streams, 1 and 3 torch streams), with the
# context's queue calibration and without it (DM_QUEUE_CALIB=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6queues}
mkdir -p $OUT
: > $OUT/queues.jsonl
for cal in 1 0; do
  for k in 0 1 2 3; do
    DM_QUEUE_CALIB=$cal timeout -k 10 120 python tools/queue_probe.py $k masked >> $OUT/queues.jsonl 2>> $OUT/err.txt || exit 1
  done
  for k in 1 3; do
    DM_QUEUE_CALIB=$cal timeout -k 10 120 python tools/queue_probe.py $k torch >> $OUT/queues.jsonl 2>> $OUT/err.txt || exit 1
  done
done
cut -c1-100 $OUT/queues.jsonl
