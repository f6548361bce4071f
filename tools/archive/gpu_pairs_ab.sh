#!/bin/bash
# GPU call: two-library C2 A/Bs in both orders (tools/gpu_r4_ab.sh) for each pair
# named in PAIRS ("tagA:libA:libB tagB:..."; libraries under tools/ab_libs).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for pr in ${PAIRS}; do
  IFS=: read -r tag a b <<< "$pr"
  WL=${WL:-c2} ROUNDS=${ROUNDS:-6} TAG=${tag}a LIBS="tools/ab_libs/$a tools/ab_libs/$b" bash tools/gpu_r4_ab.sh
  WL=${WL:-c2} ROUNDS=${ROUNDS:-6} TAG=${tag}b LIBS="tools/ab_libs/$b tools/ab_libs/$a" bash tools/gpu_r4_ab.sh
done
