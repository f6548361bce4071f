#!/bin/bash
# GPU call (round 5): the C2 tick after different preludes in one process (tools/c2_after.py);
# PRES: preludes separated by ";" (an empty one: C2 alone)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5after}
mkdir -p $OUT
i=0
IFS=';' read -ra LIST <<< "${PRES:-;c1;c3;hier;alloc;hier c1}"
for pre in "${LIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python -u tools/c2_after.py $pre > $OUT/after_$i.txt 2>&1 || { tail -5 $OUT/after_$i.txt; exit 1; }
  grep -v amdgpu.ids $OUT/after_$i.txt | tail -1
done
